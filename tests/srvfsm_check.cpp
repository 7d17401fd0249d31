// CPU unit test of the latency-mode server's host state machine (csrc/rxg_srvfsm.h) against a
// scripted device: normal service, an idle exit before a request, a kernel that never
// serves (timeout, then bounded -EIO while it stays resident, never a blocking
// synchronisation), its late exit (relaunch and service), and stop with and without a
// resident kernel.  Built and run by tests/test_srvfsm.py (also under ASan/UBSan).
#include <cassert>
#include <cerrno>
#include <chrono>
#include <cstdio>
#include <vector>

#include "rxg_srvfsm.h"

// A scripted device with a mailbox that persists across launches, like the real one: the
// last request written stays there, and a kernel starts from `done` (rx_server: last =
// ret->done) and serves any request numbered above it.
struct FakePort {
    unsigned long long done_ = 0;
    unsigned long long mbox_seq = 0;  // the request number in the mailbox
    unsigned long long last = 0;      // the resident kernel's last request seen
    bool exited_ = true;     // no kernel yet
    bool serving = true;     // a running kernel answers each request at once
    bool obeys_stop = true;  // a stop request makes it exit
    int launches = 0, syncs = 0, stops = 0, writes = 0, cancels = 0;
    bool synced_while_resident = false;
    bool exit_seen = true;   // exited() has read true since the last launch (none yet: true)
    std::vector<unsigned long long> served;  // every request a kernel served, in order

    unsigned long long done() const { return done_; }
    bool exited() const
    {
        if (exited_) const_cast<FakePort *>(this)->exit_seen = true;
        return exited_;
    }
    void serve()
    {
        if (!exited_ && serving && mbox_seq > last) {
            last = mbox_seq;
            done_ = mbox_seq;
            served.push_back(mbox_seq);
        }
    }
    void write(unsigned long long q)
    {
        ++writes;
        mbox_seq = q;
        serve();
    }
    void cancel(unsigned long long q)
    {
        assert(exited_);  // only with no kernel resident
        ++cancels;
        done_ = q;
    }
    void request_stop()
    {
        ++stops;
        if (obeys_stop) exited_ = true;
    }
    int launch()
    {
        // the Port contract: a kernel is launched only after the previous one was seen to
        // exit (or none ran), and launch() resets exited before the kernel runs
        assert(exit_seen);
        ++launches;
        exited_ = false;
        exit_seen = false;
        last = done_;
        serve();  // the new kernel polls the mailbox at once
        return 0;
    }
    void sync()
    {
        ++syncs;
        if (!exited_) synced_while_resident = true;  // would block forever on a real stream
    }
    bool was_served(unsigned long long q) const
    {
        for (auto s : served)
            if (s == q) return true;
        return false;
    }
};

using Fsm = rxg::SrvFsm<FakePort>;
using ms = std::chrono::milliseconds;

static double elapsed_ms(std::chrono::steady_clock::time_point t0)
{
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}

int main()
{
    {  // normal service: one launch, every post answered
        FakePort p;
        Fsm f;
        for (int i = 0; i < 5; ++i) assert(f.post(p) == 0);
        assert(p.launches == 1 && p.done_ == 5 && f.phase == rxg::SrvPhase::Up);
        assert(f.stop(p) == 0 && f.phase == rxg::SrvPhase::Down && p.syncs == 1);
        assert(!p.synced_while_resident);
    }
    {  // the kernel exited idle: the next post relaunches it (after synchronising it)
        FakePort p;
        Fsm f;
        assert(f.post(p) == 0);
        p.exited_ = true;  // idle exit
        assert(f.post(p) == 0 && p.launches == 2 && p.syncs == 1 && p.done_ == 2);
        assert(!p.synced_while_resident);
    }
    {  // a kernel that never serves and ignores stop: -ETIMEDOUT, then bounded -EIO
        FakePort p;
        Fsm f;
        f.serve_timeout = ms(30);
        f.exit_timeout = ms(20);
        assert(f.post(p) == 0);
        p.serving = false;
        p.obeys_stop = false;
        auto t0 = std::chrono::steady_clock::now();
        assert(f.post(p) == -ETIMEDOUT);
        assert(elapsed_ms(t0) < 2000.0);
        assert(f.phase == rxg::SrvPhase::Failed && p.stops == 1);
        const int writes = p.writes, launches = p.launches;
        for (int i = 0; i < 3; ++i) {
            t0 = std::chrono::steady_clock::now();
            assert(f.post(p) == -EIO);  // waits at most exit_timeout, posts nothing
            assert(elapsed_ms(t0) < 1000.0);
        }
        assert(p.writes == writes && p.launches == launches);
        t0 = std::chrono::steady_clock::now();
        assert(f.stop(p) == -EIO && elapsed_ms(t0) < 1000.0 && f.phase == rxg::SrvPhase::Failed);
        assert(!p.synced_while_resident);
        // the kernel finally leaves: the next post synchronises, relaunches and is served
        p.exited_ = true;
        p.serving = true;
        p.obeys_stop = true;
        const unsigned long long timed_out = f.seq - 0;  // the request that failed, still in the mailbox
        assert(p.mbox_seq == timed_out && !p.was_served(timed_out));
        assert(f.post(p) == 0 && f.phase == rxg::SrvPhase::Up && p.launches == launches + 1);
        assert(p.done_ == f.seq && p.cancels == 1);
        // the relaunched kernel served the new request only, never the
        // one whose caller was told -ETIMEDOUT
        assert(!p.was_served(timed_out));
        assert(p.served.back() == f.seq);
        assert(f.stop(p) == 0 && f.phase == rxg::SrvPhase::Down);
        assert(!p.synced_while_resident);
    }
    {  // a timed-out kernel that does obey stop: the next post relaunches at once
        FakePort p;
        Fsm f;
        f.serve_timeout = ms(10);
        assert(f.post(p) == 0);
        p.serving = false;
        assert(f.post(p) == -ETIMEDOUT && p.exited_);
        const unsigned long long timed_out = f.seq;
        p.serving = true;
        assert(f.post(p) == 0 && p.launches == 2);
        assert(!p.was_served(timed_out) && p.served.back() == f.seq);
        assert(!p.synced_while_resident);
    }
    {  // the mailbox persists: after a timeout, two more posts, each served exactly once
        FakePort p;
        Fsm f;
        f.serve_timeout = ms(10);
        assert(f.post(p) == 0 && f.post(p) == 0);
        p.serving = false;
        assert(f.post(p) == -ETIMEDOUT);
        const unsigned long long timed_out = f.seq;
        p.serving = true;
        assert(f.post(p) == 0 && f.post(p) == 0);
        const std::vector<unsigned long long> want = {1, 2, timed_out + 1, timed_out + 2};
        assert(p.served == want);
        assert(!p.synced_while_resident);
    }
    {  // an idle exit is not a failure: the request posted to the exited kernel is served by
       // the relaunched one (no cancel)
        FakePort p;
        Fsm f;
        assert(f.post(p) == 0);
        p.exited_ = true;  // idle exit, unobserved until the next post
        assert(f.post(p) == 0 && p.cancels == 0 && p.served.back() == f.seq);
    }
    {  // stop with nothing launched
        FakePort p;
        Fsm f;
        assert(f.stop(p) == 0 && p.stops == 0);
    }
    std::puts("srvfsm ok");
    return 0;
}
