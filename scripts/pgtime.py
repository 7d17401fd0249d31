#!/usr/bin/env python3
"""Time rxg_payload_gather_dev over the bench's C3 / C4 batch (one rx burst, then N gathers
into an arena of exactly the burst's size), median of HIP events around each gather.  With
RXG_LIB_OVERRIDE=1 RXG_LIB=<path> it times another build of the library: run the two builds
alternately in separate processes for an A/B on one box.
  python scripts/pgtime.py [--workload c3|c4] [--iters 30]"""
import argparse
import json
import os
import sys

import numpy as np
import torch  # noqa: F401  (one HIP runtime per process)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dpdk-tcpipstack_amd")]
import rxg  # noqa: E402

WL = {"c3": (1500, 1000, 0), "c4": (0, 65536, 1)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="c3", choices=sorted(WL))
    ap.add_argument("--iters", type=int, default=30)
    args = ap.parse_args()
    L, flows, mix = WL[args.workload]
    n = 1 << 20
    eng = rxg.Engine(0)
    b = eng.synth(n=n, nflows=flows, len_a=L or 1500, mix=mix, seed=0x5EED0001)
    eng.tcb_load(*rxg.synthetic_tcb_table(flows))
    out = eng.alloc(n * 8)
    eng.rx_burst_dev(b["arena"].ptr, b["off64"].ptr, b["len"].ptr, n, out.ptr, 8)
    pl = (b["len"].download(np.uint16, n).astype(np.int64) - 54).clip(min=0)
    cap = int(((pl + 15) // 16 * 16).sum())
    arena, msgs, used = eng.alloc(cap), eng.alloc(n * 16), eng.alloc(8)
    ev = [(eng.event(), eng.event()) for _ in range(args.iters)]
    for _ in range(3):
        eng.payload_gather_dev(arena.ptr, cap, msgs.ptr, used.ptr)
    for e0, e1 in ev:
        eng.record(e0)
        eng.payload_gather_dev(arena.ptr, cap, msgs.ptr, used.ptr)
        eng.record(e1)
    eng.sync()
    us = sorted(eng.elapsed_ms(e0, e1) * 1e3 for e0, e1 in ev)
    assert int(used.download(np.uint64, 1)[0]) == cap
    print(json.dumps({"workload": args.workload, "lib": rxg.build_provenance()["build"],
                      "us_median": round(us[len(us) // 2], 2), "us_min": round(us[0], 2)}), flush=True)


if __name__ == "__main__":
    main()
