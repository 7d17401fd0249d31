// rxg_srvfsm.h — the host side of the latency-mode server's protocol (rxg_server_*, DESIGN.md
// §2.5) as a state machine over a Port, so its failure paths run in a CPU unit test
// (tests/srvfsm_check.cpp) with a scripted device instead of a GPU.
//
// Port (rxg_server.cpp: the real mailbox, return block and stream):
//   unsigned long long done()    the number of the last request the server finished
//   bool exited()                the kernel has left its loop (stop or idle)
//   void write(q)                post request number q (mailbox words; the request body is
//                                the port's business)
//   void cancel(q)               no kernel is resident: make request q (still in the mailbox)
//                                one the next kernel will not serve (its `done` reads q)
//   void request_stop()          ask the kernel to leave its loop
//   int  launch()                start a kernel (the previous one has exited or none ran;
//                                its stream is synchronised first): 0 or a negative errno.
//                                It resets exited() to false BEFORE the kernel starts: the
//                                machine synchronises a stream on the strength of exited()
//                                alone (tests/srvfsm_check.cpp holds it to that)
//   void sync()                  wait for the exited kernel's stream (returns at once: the
//                                kernel has left its loop)
//
// Phases: Down (no kernel launched since the last synchronisation), Up, Failed (a request was
// not served in time; a stop was requested, but the kernel may still be resident and may
// still write the shared staging and records).  A Failed server is reused only after its
// kernel has exited, which each call waits for at most exit_timeout, else it returns -EIO:
// no call ever blocks on a stream synchronisation with a kernel that has not exited.
#pragma once
#include <cerrno>
#include <chrono>

namespace rxg {

enum class SrvPhase { Down, Up, Failed };

template <class Port>
struct SrvFsm {
    using clock = std::chrono::steady_clock;
    SrvPhase phase = SrvPhase::Down;
    unsigned long long seq = 0;  // the last request number posted
    std::chrono::nanoseconds serve_timeout = std::chrono::seconds(10);
    std::chrono::nanoseconds exit_timeout = std::chrono::seconds(1);

    // spin until the kernel has exited, at most `limit`
    static bool wait_exited(Port &p, std::chrono::nanoseconds limit)
    {
        const auto t0 = clock::now();
        for (unsigned spins = 0; !p.exited(); ++spins) {
            if ((spins & 255u) == 0u && clock::now() - t0 > limit) return false;
            pause();
        }
        return true;
    }

    // a kernel that exited (idle, or stopped) is synchronised and relaunched
    int relaunch(Port &p)
    {
        if (phase != SrvPhase::Down) p.sync();
        phase = SrvPhase::Down;
        const int rc = p.launch();
        if (rc) return rc;
        phase = SrvPhase::Up;
        return 0;
    }

    // A kernel ready to serve: -EIO while a failed kernel is still resident.  Relaunching
    // after a failure first cancels the request that timed out: its caller was told it
    // failed (and may have freed its output), so no later kernel may serve it.
    int ready(Port &p)
    {
        if (phase == SrvPhase::Failed) {
            if (!wait_exited(p, exit_timeout)) return -EIO;
            p.sync();
            phase = SrvPhase::Down;
            p.cancel(seq);
            return relaunch(p);
        }
        if (phase == SrvPhase::Down || p.exited()) return relaunch(p);
        return 0;
    }

    // Post one request and wait for its `done`.  A kernel that exited idle before it saw the
    // request is relaunched; the new one starts from `done` and serves it.
    int post(Port &p)
    {
        int rc = ready(p);
        if (rc) return rc;
        const unsigned long long q = ++seq;
        p.write(q);
        const auto t0 = clock::now();
        for (unsigned long long spins = 1;; ++spins) {
            if (p.done() == q) return 0;
            pause();
            if ((spins & 1023u) == 0u) {
                if (p.exited()) {
                    if (p.done() == q) return 0;
                    if ((rc = relaunch(p))) return rc;
                }
                if (clock::now() - t0 > serve_timeout) {
                    p.request_stop();
                    phase = SrvPhase::Failed;
                    return -ETIMEDOUT;
                }
            }
        }
    }

    // Stop: 0 once the kernel has exited (or none runs); -EIO (phase Failed) if it has not
    // within exit_timeout.
    int stop(Port &p)
    {
        if (phase == SrvPhase::Down) return 0;
        p.request_stop();
        if (!wait_exited(p, exit_timeout)) {
            phase = SrvPhase::Failed;
            return -EIO;
        }
        p.sync();
        phase = SrvPhase::Down;
        return 0;
    }

    static void pause()
    {
#if defined(__x86_64__)
        __builtin_ia32_pause();
#endif
    }
};

}  // namespace rxg
