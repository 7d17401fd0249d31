#!/usr/bin/env python3
"""Grid-cap sensitivity of the rx kernel (rxg_config.max_blocks): one engine per cap in one
process, the bench's C3 / C4 / C2 batches (rotating copies), interleaved rounds, median of
HIP-event time per launch over a block of back-to-back launches.
  python scripts/gridbench.py [--caps 0,512,768,1024] [--rounds 5]"""
import argparse
import json
import os
import sys

import numpy as np
import torch  # noqa: F401  (one HIP runtime per process)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dpdk-tcpipstack_amd")]
import rxg  # noqa: E402

WL = {"c3": (1500, 1000, 0, 2), "c4": (0, 65536, 1, 3), "c2": (64, 1, 0, 16)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--caps", default="0,512,768,1024")
    ap.add_argument("--workloads", default="c3,c4,c2")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=20)
    args = ap.parse_args()
    caps = [int(x) for x in args.caps.split(",")]
    n = 1 << 20
    engs = {c: rxg.Engine(0, max_blocks=c) for c in caps}
    res = {}
    for w in args.workloads.split(","):
        L, flows, mix, copies = WL[w]
        e0 = engs[caps[0]]
        bs = [e0.synth(n=n, nflows=flows, len_a=L or 1500, mix=mix, seed=0x5EED0001 + 17 * c) for c in range(copies)]
        for e in engs.values():
            e.tcb_load(*rxg.synthetic_tcb_table(flows))
        out = e0.alloc(n * 8)
        t = {c: [] for c in caps}
        for _ in range(args.rounds):
            for c, e in engs.items():
                a, b = e.event(), e.event()
                for i in range(3):
                    x = bs[i % copies]
                    e.rx_burst_dev(x["arena"].ptr, x["off64"].ptr, x["len"].ptr, n, out.ptr, 8)
                e.record(a)
                for i in range(args.iters):
                    x = bs[i % copies]
                    e.rx_burst_dev(x["arena"].ptr, x["off64"].ptr, x["len"].ptr, n, out.ptr, 8)
                e.record(b)
                e.sync()
                t[c].append(e.elapsed_ms(a, b) * 1e3 / args.iters)
        res[w] = {str(c): round(float(np.median(v)), 2) for c, v in t.items()}
        print(json.dumps({"workload": w, "us_per_launch_median": res[w]}), flush=True)
        out.free()
        for x in bs:
            for v in x.values():
                if isinstance(v, rxg.DevArray):
                    v.free()


if __name__ == "__main__":
    main()
