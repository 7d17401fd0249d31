#!/usr/bin/env python3
"""Host-burst latency: rxg_rx_burst (host mbuf views -> pinned staging -> H2D -> kernel ->
D2H records, synchronous) at burst sizes around the reference's MAX_PKT_BURST = 32
(main.c:116), plus rxg_ether_in (one frame per call) and rxg_rx_replay with empty
handlers.  Views are built once; the timed loop is the C calls only.
  python scripts/latbench.py [sizes...]"""
import ctypes as C
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dpdk-tcpipstack_amd"), os.path.join(ROOT, "tests")]
import torch  # noqa: E402,F401
import pktgen  # noqa: E402
import rxg  # noqa: E402


def main():
    sizes = [int(x) for x in (sys.argv[1:] or ["1", "32", "256", "1024", "4096", "65536"])]
    eng = rxg.Engine(0, max_batch=max(sizes), max_bytes=max(sizes) * 1536)
    lib = rxg.load_library()
    tcb, live = rxg.synthetic_tcb_table(1000)
    eng.tcb_load(tcb, live)
    dst = pktgen.ip4(192, 168, 78, 2)
    frames = [pktgen.frame(src_ip=(10 << 24) | (f % 1000), dst_ip=dst, sport=1024 + f % 1000, dport=80,
                           payload=bytes(1446)) for f in range(max(sizes))]
    bufs = [C.create_string_buffer(f, len(f)) for f in frames]
    views = (rxg.PktView * len(frames))(*[rxg.PktView(C.addressof(b), 0, len(f), 0) for b, f in zip(bufs, frames)])
    out = np.zeros(max(sizes), dtype=rxg.REC16_DTYPE)
    out_p = out.ctypes.data  # once: numpy's .ctypes.data costs ~2 us per access in Python
    ptrs = (C.c_void_p * len(bufs))(*[C.addressof(b) for b in bufs])
    ops = rxg.HandoffOps()
    for n in sizes:
        iters = max(20, min(2000, 200000 // n))
        for _ in range(5):
            lib.rxg_rx_burst(eng.ctx, views, n, rxg.REC16, out_p)
        t0 = time.perf_counter()
        for _ in range(iters):
            rc = lib.rxg_rx_burst(eng.ctx, views, n, rxg.REC16, out_p)
        dt = (time.perf_counter() - t0) / iters
        assert rc == 0
        t0 = time.perf_counter()
        for _ in range(iters):
            lib.rxg_rx_burst(eng.ctx, views, n, rxg.REC16, out_p)
            lib.rxg_rx_replay(eng.ctx, C.byref(ops), ptrs, ptrs, out_p, n, rxg.REC16)
        dr = (time.perf_counter() - t0) / iters
        print(json.dumps({"burst": n, "rx_burst_us": round(dt * 1e6, 1), "mpps": round(n / dt / 1e6, 3),
                          "burst_plus_replay_us": round(dr * 1e6, 1)}), flush=True)
    t0 = time.perf_counter()
    for i in range(500):
        lib.rxg_ether_in(eng.ctx, C.byref(ops), ptrs[i % len(bufs)], ptrs[i % len(bufs)], len(frames[0]))
    print(json.dumps({"ether_in_us": round((time.perf_counter() - t0) / 500 * 1e6, 1)}), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
