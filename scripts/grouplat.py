#!/usr/bin/env python3
"""Group burst latency: rxg_group_rx_burst on a 2-member group (both
members on the box's one GPU: two contexts, two streams, the group's persistent worker
thread) against one context's rxg_rx_burst, at 32 and 4 096 host frames of 1 500 B; and the
device-resident group burst (rxg_group_rx_burst_dev + rxg_group_sync) at the same sizes.
  python scripts/grouplat.py"""
import ctypes as C
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dpdk-tcpipstack_amd")]
import torch  # noqa: E402,F401
import rxg  # noqa: E402


def timed(fn, budget=0.5):
    for _ in range(5):
        fn()
    it, t0 = 0, time.perf_counter()
    while True:
        fn()
        it += 1
        dt = time.perf_counter() - t0
        if dt > budget and it >= 10:
            return round(dt / it * 1e6, 1)


def main():
    nmax = 4096
    lib = rxg.load_library()
    eng = rxg.Engine(0, max_batch=nmax, max_bytes=nmax * 1536)
    b = eng.synth(n=nmax, nflows=1000, len_a=1500, seed=5)
    eng.sync()
    off = b["off64"].download(np.uint32, nmax)
    lens = b["len"].download(np.uint16, nmax)
    arena = b["arena"].download(np.uint8, b["arena_bytes"])
    tcb, live = rxg.synthetic_tcb_table(1000)
    eng.tcb_load(tcb, live)
    base = arena.ctypes.data
    views = (rxg.PktView * nmax)(*[rxg.PktView(base + int(o) * 64, 0, int(ln), 0) for o, ln in zip(off, lens)])
    out = np.zeros(nmax, dtype=rxg.REC8_DTYPE)
    out_p = out.ctypes.data  # once: numpy's .ctypes.data costs ~2 us per access in Python
    res = {}
    with rxg.Group([0, 0], max_batch=nmax, max_bytes=nmax * 1536) as g:
        g.tcb_load(tcb, live)
        dev = []
        for n in (32, 4096):
            res[f"single_ctx_rx_burst_{n}_us"] = timed(lambda: lib.rxg_rx_burst(eng.ctx, views, n, rxg.REC8, out_p))
            res[f"group2_rx_burst_{n}_us"] = timed(lambda: lib.rxg_group_rx_burst(g.g, views, n, rxg.REC8, out_p))
            # device-resident: each member's half already in device memory (the same device here)
            half = n // 2
            shards = []
            for i, m in enumerate(g.members):
                lo, hi = i * half, (i + 1) * half
                da = b["arena"].ptr
                do = m.to_device(np.ascontiguousarray(off[lo:hi]))
                dl = m.to_device(np.ascontiguousarray(lens[lo:hi]))
                dout = m.alloc(half * 8)
                dev += [do, dl, dout]
                shards.append(rxg.DevBatch(da, do.ptr, dl.ptr, half, rxg.REC8, dout.ptr))
            arr = (rxg.DevBatch * 2)(*shards)

            def devburst():
                assert lib.rxg_group_rx_burst_dev(g.g, arr, 2) == 0
                assert lib.rxg_group_sync(g.g) == 0
            res[f"group2_rx_burst_dev_{n}_us"] = timed(devburst)
            dsingle = eng.alloc(n * 8)
            single = rxg.DevBatch(b["arena"].ptr, b["off64"].ptr, b["len"].ptr, n, rxg.REC8, dsingle.ptr)

            def devsingle():
                assert lib.rxg_rx_burst_dev(eng.ctx, C.byref(single), None) == 0
                assert lib.rxg_sync(eng.ctx) == 0
            res[f"single_ctx_rx_burst_dev_{n}_us"] = timed(devsingle)
            dsingle.free()
        for d in dev:
            d.free()
    print(json.dumps({"group_latency": res, "frames": "1500 B, 1000 flows, REC8",
                      "note": "both group members on one GPU: the group's host path and concurrency, not two GPUs"}))
    eng.close()


if __name__ == "__main__":
    main()
