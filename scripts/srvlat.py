#!/usr/bin/env python3
"""Latency-mode breakdown (rxg_server_*): where a small burst's microseconds go.

  launched   rxg_rx_burst (zero-copy launch + stream sync) + rxg_rx_replay, empty handlers
  served     the same through the server
  served-nr  the server, burst only (no replay)
  dev-1      rxg_server_burst_dev of ONE device-resident frame: the mailbox round trip floor
  dev-n      rxg_server_burst_dev of the burst's frames resident in HBM (no PCIe frame reads)

The served columns are measured for both placements of the mailbox and staging, one after
the other in the same process: "device" staging (device memory the host writes through the
BAR, the default on a large-BAR GPU), "_hostmem" (RXG_SRV_HOST_STAGING, coherent host memory)
and "_hostmbox" (RXG_SRV_HOST_MAILBOX: device staging, the mailbox in host memory).

python scripts/srvlat.py [--blocks 4]   (one JSON line per frame size and burst)"""
import argparse
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


def per_call_us(fn, budget=0.3):
    for _ in range(5):
        fn()
    it, t0 = 0, time.perf_counter()
    lat = []
    while True:
        a = time.perf_counter()
        fn()
        lat.append(time.perf_counter() - a)
        it += 1
        if time.perf_counter() - t0 > budget and it >= 20:
            return round(float(np.median(lat)) * 1e6, 2)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--blocks", type=int, default=4)
    args = ap.parse_args()
    nmax = 4096
    eng = rxg.Engine(0, max_batch=nmax, max_bytes=nmax * 1536)
    lib = rxg.load_library()
    out = np.zeros(nmax, dtype=rxg.REC8_DTYPE)
    out_p = out.ctypes.data  # once: numpy's .ctypes.data costs ~2 us per access in Python
    ops = rxg.HandoffOps()
    ops_r = C.byref(ops)
    for size in (64, 1500):
        b = eng.synth(n=nmax, nflows=1000, len_a=size, seed=99)
        eng.sync()
        off = b["off64"].download(np.uint32, nmax)
        lens = b["len"].download(np.uint16, nmax)
        arena = b["arena"].download(np.uint8, b["arena_bytes"])
        tcb, live = rxg.synthetic_tcb_table(1000)
        eng.tcb_load(tcb, live)
        base = arena.ctypes.data
        views = (rxg.PktView * nmax)(*[rxg.PktView(base + int(o) * 64, 0, int(ln), 0) for o, ln in zip(off, lens)])
        ptrs = (C.c_void_p * nmax)(*[base + int(o) * 64 for o in off])
        d_out = eng.alloc(nmax * 8)
        for n in (1, 32, 256):
            def burst():
                assert lib.rxg_rx_burst(eng.ctx, views, n, rxg.REC8, out_p) == 0

            def burst_replay():
                burst()
                assert lib.rxg_rx_replay(eng.ctx, ops_r, ptrs, ptrs, out_p, n, rxg.REC8) == 0

            dbatch = rxg.DevBatch(b["arena"].ptr, b["off64"].ptr, b["len"].ptr, n, rxg.REC8, d_out.ptr)
            dref = C.byref(dbatch)  # built once, as the C loop would

            def dev():
                assert lib.rxg_server_burst_dev(eng.ctx, dref) == 0
            row = {"frame_bytes": size, "n": n, "launched": per_call_us(burst_replay),
                   "launched_nr": per_call_us(burst)}
            for tag, flags in (("", 0), ("_hostmem", rxg.SRV_HOST_STAGING), ("_hostmbox", rxg.SRV_HOST_MAILBOX)):
                eng.server_start(rxg.REC8, blocks=args.blocks, max_frames=nmax, flags=flags)
                row["placement" + tag] = {rxg.SRV_DEVICE: "device", rxg.SRV_HOST: "host"}[eng.server_placement()]
                row.update({"served" + tag: per_call_us(burst_replay), "served_nr" + tag: per_call_us(burst),
                            "dev" + tag: per_call_us(dev)})
                eng.server_stop()
            print(json.dumps(row), flush=True)
        d_out.free()
        for v in b.values():
            if isinstance(v, rxg.DevArray):
                v.free()
    eng.close()


if __name__ == "__main__":
    main()
