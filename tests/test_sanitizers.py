"""CPU: the host code under AddressSanitizer + UndefinedBehaviorSanitizer (SURVEY.md §5,
"race detection / sanitizers"); ThreadSanitizer runs stay in tests/test_opqueue.py.

  * the TCB / ARP mirror (csrc/rxg_mirror.h: backward-shift deletion, duplicate tuples,
    rebuilds) driven by tests/mirror_check.cpp against a naive two-pass findtcb;
  * the packing / group worker pool (csrc/rxg_packpool.h) and the cross-thread post queue
    (csrc/rxg_opqueue.h);
  * the oracle (oracle/rxg_oracle.c) over frames in exact-size heap blocks
    (tests/sanitize_oracle.c): its handling of the reference's over-reads is checked, not
    assumed.

Every build uses -fno-sanitize-recover=all, so any report fails the run.  Host code only
(no GPU): the sanitizers are built with g++/gcc for the host, never into a GPU code object.
"""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "dpdk-tcpipstack_amd", "csrc")
BUILD = os.path.join(ROOT, "build_abi_probe", "san")
SAN = ["-fsanitize=address,undefined", "-fno-sanitize-recover=all", "-fno-omit-frame-pointer", "-g", "-O1"]
ENV = {**os.environ, "ASAN_OPTIONS": "detect_leaks=1:abort_on_error=0:halt_on_error=1",
       "UBSAN_OPTIONS": "halt_on_error=1:print_stacktrace=1"}

pytestmark = pytest.mark.skipif(shutil.which("g++") is None or shutil.which("gcc") is None,
                                reason="gcc/g++ missing")


def _build(cmd, exe):
    os.makedirs(BUILD, exist_ok=True)
    r = subprocess.run(cmd + ["-o", exe], capture_output=True, text=True)
    if r.returncode != 0 and "sanitize" in r.stderr and "cannot find" in r.stderr:
        pytest.skip("toolchain without ASan/UBSan runtimes")
    assert r.returncode == 0, r.stderr[-3000:]
    return exe


def _run(args, timeout=600):
    r = subprocess.run(args, capture_output=True, text=True, timeout=timeout, env=ENV)
    assert r.returncode == 0 and "ERROR: AddressSanitizer" not in r.stderr and "runtime error" not in r.stderr, \
        (r.stdout + r.stderr)[-4000:]
    return r.stdout


@pytest.fixture(scope="module")
def mirror_exe():
    return _build(["g++", "-std=c++17", *SAN, "-D__HIP_PLATFORM_AMD__", "-I/opt/rocm/include",
                   "-I", os.path.join(ROOT, "include"), "-I", CSRC, os.path.join(ROOT, "tests", "mirror_check.cpp")],
                  os.path.join(BUILD, "mirror_check_asan"))


@pytest.mark.parametrize("seed,ops,keys", [(11, 20000, 40), (12, 20000, 400), (13, 30000, 5000), (14, 4000, 3),
                                            (15, 12000, 100000)])
def test_mirror_under_asan_ubsan(mirror_exe, seed, ops, keys):
    out = _run([mirror_exe, str(seed), str(ops), str(keys)])
    assert out.startswith("ok"), out


@pytest.fixture(scope="module")
def oracle_exe():
    return _build(["gcc", "-std=c11", *SAN, "-Wall", "-Wextra", "-Werror", "-I", os.path.join(ROOT, "include"),
                   os.path.join(ROOT, "tests", "sanitize_oracle.c"), os.path.join(ROOT, "oracle", "rxg_oracle.c")],
                  os.path.join(BUILD, "sanitize_oracle"))


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_oracle_under_asan_ubsan(oracle_exe, seed):
    out = _run([oracle_exe, str(seed), "20000"])
    assert out.startswith("ok"), out


def test_oracle_asan_catches_an_over_read(tmp_path):
    """The harness would see the reference's over-read: a checksum over an odd span whose
    byte after it is not allocated is an ASan report (the oracle's callers never do this)."""
    src = tmp_path / "over.c"
    src.write_text('#include <stdlib.h>\n#include <string.h>\n#include "../oracle/rxg_oracle.h"\n'
                   'int main(void){ unsigned char *p = malloc(21); memset(p, 1, 21);\n'
                   '  int r = orc_calculate_checksum(p, 21); free(p); return r == 0x1234; }\n')
    exe = _build(["gcc", "-std=c11", *SAN, "-I", os.path.join(ROOT, "include"), "-I", os.path.join(ROOT, "tests"),
                  str(src), os.path.join(ROOT, "oracle", "rxg_oracle.c")], str(tmp_path / "over"))
    r = subprocess.run([exe], capture_output=True, text=True, timeout=60, env=ENV)
    assert r.returncode != 0 and "heap-buffer-overflow" in r.stderr


POOL_AND_QUEUE = r'''
#include <cstdio>
#include <thread>
#include <vector>
#include "rxg_opqueue.h"
#include "rxg_packpool.h"

struct Op { unsigned producer, seq; };

int main() {
    {   // the pool: jobs split 1..8 ways back to back, every index exactly once
        rxg::PackPool pool;
        std::vector<int> hits(1 << 14);
        for (int round = 0; round < 1500; ++round) {
            const unsigned n = 1u + (unsigned)(round * 7 % 8);
            const size_t m = hits.size();
            pool.run(n, [&](unsigned t) {
                for (size_t i = m * t / n; i < m * (t + 1) / n; ++i) hits[i] += 1;
            });
            for (size_t i = 0; i < m; ++i)
                if (hits[i] != round + 1) { std::printf("FAIL pool round %d index %zu\n", round, i); return 1; }
        }
    }
    {   // the post queue: 4 producers, one consumer, exactly once and in order per producer
        const unsigned P = 4, N = 50000;
        rxg::MpscRing<Op> q(256);
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
            if (o.producer >= P || o.seq != next[o.producer]) { std::printf("FAIL queue\n"); return 1; }
            ++next[o.producer];
            ++got;
        }
        for (auto &t : th) t.join();
    }
    std::printf("ok\n");
    return 0;
}
'''


def test_pool_and_queue_under_asan_ubsan():
    os.makedirs(BUILD, exist_ok=True)
    src = os.path.join(BUILD, "pool_queue_asan.cpp")
    with open(src, "w") as fh:
        fh.write(POOL_AND_QUEUE)
    exe = _build(["g++", "-std=c++17", *SAN, "-pthread", "-I", CSRC, src], os.path.join(BUILD, "pool_queue_asan"))
    assert _run([exe]).startswith("ok")
