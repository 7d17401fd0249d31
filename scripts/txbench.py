#!/usr/bin/env python3
"""Tx checksum-generate micro-benchmark: rxg_tx_cksum_dev over the C3 / C4 batch, one rxg
context per grid cap (rxg_config.max_blocks) (0 = occupancy grid), interleaved rounds.
  python scripts/txbench.py --grids 0,768 --workloads c3,c4
A grid may name another librxg build as GRID:PATH (A/B of two builds in one process)."""
import argparse
import json
import os
import sys

import numpy as np
import torch  # noqa: F401  (one HIP runtime per process)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dpdk-tcpipstack_amd")]
import rxg  # noqa: E402

WL = {"c3": (1500, 0), "c4": (0, 1), "c2": (64, 0)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--grids", default="0")
    ap.add_argument("--workloads", default="c3,c4")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--iters", type=int, default=10)
    args = ap.parse_args()
    engs, libs = {}, {}
    main_lib = rxg.load_library()
    for g in args.grids.split(","):
        grid, _, path = g.partition(":")
        lib = main_lib
        if path:
            rxg._lib = None
            lib = rxg.load_library(path)
        rxg._lib = lib
        libs[g] = lib
        engs[g] = rxg.Engine(0, max_blocks=int(grid or 0))
        rxg._lib = main_lib
    base = engs[args.grids.split(",")[0]]
    rxg._lib = libs[args.grids.split(",")[0]]
    n = 1 << 20
    res = {}
    for w in args.workloads.split(","):
        L, mix = WL[w]
        b = base.synth(n=n, nflows=1000, len_a=L or 1500, mix=mix, seed=9)
        nbytes = int(b["len"].download(np.uint16, n).astype(np.int64).sum())
        for r in range(args.rounds):
            for g, eng in engs.items():
                rxg._lib = libs[g]
                evs = [(eng.event(), eng.event()) for _ in range(args.iters)]
                eng.tx_cksum_dev(b["arena"].ptr, b["off64"].ptr, b["len"].ptr, n)
                for a, e in evs:
                    eng.record(a)
                    eng.tx_cksum_dev(b["arena"].ptr, b["off64"].ptr, b["len"].ptr, n)
                    eng.record(e)
                eng.sync()
                res.setdefault((g, w), []).append(float(np.median([eng.elapsed_ms(a, e) for a, e in evs])))
        res[("bytes", w)] = nbytes
    for (g, w), ms in res.items():
        if g == "bytes":
            continue
        med = float(np.median(ms))
        nb = res[("bytes", w)]
        print(json.dumps({"grid": g, "workload": w, "kernel_us": round(med * 1e3, 2),
                          "frac_8TBs": round(nb / (med * 1e-3) / 8e12, 4)}), flush=True)


if __name__ == "__main__":
    main()
