"""CPU tests of the host-side concurrency pieces, built with ThreadSanitizer when the
toolchain has it:
  - the cross-thread TCB-mirror queue (csrc/rxg_opqueue.h, behind rxg_tcb_post): several
    producer threads push numbered ops while one consumer pops concurrently; every op
    arrives exactly once and each producer's ops arrive in its posting order;
  - the packing pool (csrc/rxg_packpool.h, behind rxg_rx_burst): jobs split 1..8 ways, run
    back to back, cover every index exactly once."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "dpdk-tcpipstack_amd", "csrc")
BUILD = os.path.join(ROOT, "build_abi_probe")

STRESS = r'''
#include <cstdio>
#include <thread>
#include <vector>
#include "rxg_opqueue.h"

struct Op { unsigned producer, seq; };

int main(int argc, char **argv) {
    const unsigned P = 4, N = 200000;
    rxg::MpscRing<Op> q(1024);           // small: producers meet a full ring often
    std::vector<std::thread> th;
    for (unsigned p = 0; p < P; ++p)
        th.emplace_back([&, p] {
            for (unsigned i = 0; i < N; ++i)
                while (!q.push(Op{p, i})) std::this_thread::yield();
        });
    std::vector<unsigned> next(P, 0);
    unsigned long got = 0;
    while (got < (unsigned long)P * N) {
        Op o;
        if (!q.pop(o)) { std::this_thread::yield(); continue; }
        if (o.producer >= P || o.seq != next[o.producer]) {
            std::printf("FAIL producer %u seq %u expected %u\n", o.producer, o.seq,
                        o.producer < P ? next[o.producer] : 0u);
            return 1;
        }
        ++next[o.producer];
        ++got;
    }
    for (auto &t : th) t.join();
    Op o;
    if (q.pop(o)) { std::printf("FAIL extra op\n"); return 1; }
    std::printf("OK %lu\n", got);
    return 0;
}
'''


def _build(extra):
    os.makedirs(BUILD, exist_ok=True)
    src = os.path.join(BUILD, "opqueue_stress.cpp")
    exe = os.path.join(BUILD, "opqueue_stress" + ("_tsan" if extra else ""))
    with open(src, "w") as fh:
        fh.write(STRESS)
    r = subprocess.run(["g++", "-std=c++17", "-O2", "-pthread", *extra, "-I", CSRC, src, "-o", exe],
                       capture_output=True, text=True)
    return exe if r.returncode == 0 else None


def test_mpsc_ring_order_and_exactly_once():
    exe = _build([])
    assert exe, "g++ failed on rxg_opqueue.h"
    out = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0 and out.stdout.startswith("OK 800000"), out.stdout + out.stderr


def test_mpsc_ring_under_thread_sanitizer():
    exe = _build(["-fsanitize=thread", "-g"])
    if exe is None:
        pytest.skip("g++ without ThreadSanitizer")
    out = subprocess.run([exe], capture_output=True, text=True, timeout=300,
                         env={**os.environ, "TSAN_OPTIONS": "halt_on_error=1"})
    if "FATAL: ThreadSanitizer" in out.stderr and "unexpected memory mapping" in out.stderr:
        pytest.skip("ThreadSanitizer cannot run in this container")
    assert out.returncode == 0 and "WARNING: ThreadSanitizer" not in out.stderr, out.stdout + out.stderr[-2000:]


POOL = r'''
#include <atomic>
#include <cstdio>
#include <vector>
#include "rxg_packpool.h"

int main() {
    rxg::PackPool pool;
    std::vector<int> hits(1 << 16);
    for (int round = 0; round < 3000; ++round) {
        const unsigned n = 1u + (unsigned)(round * 7 % 8);
        const size_t m = hits.size();
        pool.run(n, [&](unsigned t) {
            for (size_t i = m * t / n; i < m * (t + 1) / n; ++i) hits[i] += 1;
        });
        for (size_t i = 0; i < m; ++i)
            if (hits[i] != round + 1) { std::printf("FAIL round %d index %zu\n", round, i); return 1; }
    }
    std::printf("OK\n");
    return 0;
}
'''


def _build_pool(extra):
    os.makedirs(BUILD, exist_ok=True)
    src = os.path.join(BUILD, "packpool_check.cpp")
    exe = os.path.join(BUILD, "packpool_check" + ("_tsan" if extra else ""))
    with open(src, "w") as fh:
        fh.write(POOL)
    r = subprocess.run(["g++", "-std=c++17", "-O2", "-pthread", *extra, "-I", CSRC, src, "-o", exe],
                       capture_output=True, text=True)
    return exe if r.returncode == 0 else None


def test_packing_pool_covers_every_index_once():
    exe = _build_pool([])
    assert exe, "g++ failed on rxg_packpool.h"
    out = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0 and out.stdout.startswith("OK"), out.stdout + out.stderr


def test_packing_pool_under_thread_sanitizer():
    exe = _build_pool(["-fsanitize=thread", "-g"])
    if exe is None:
        pytest.skip("g++ without ThreadSanitizer")
    out = subprocess.run([exe], capture_output=True, text=True, timeout=300,
                         env={**os.environ, "TSAN_OPTIONS": "halt_on_error=1"})
    if "FATAL: ThreadSanitizer" in out.stderr and "unexpected memory mapping" in out.stderr:
        pytest.skip("ThreadSanitizer cannot run in this container")
    assert out.returncode == 0 and "WARNING: ThreadSanitizer" not in out.stderr, out.stdout + out.stderr[-2000:]
