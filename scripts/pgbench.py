#!/usr/bin/env python3
"""Payload-gather micro-benchmark (rxg_payload_gather_dev after one rx burst):
  python scripts/pgbench.py --workloads c3,c4,c2 --iters 20"""
import argparse
import json
import os
import sys

import numpy as np
import torch  # noqa: F401  (one HIP runtime per process)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dpdk-tcpipstack_amd")]
# the experiment library (make -C dpdk-tcpipstack_amd experiments): the variant switches
os.environ.setdefault("RXG_LIB", os.path.join(ROOT, "dpdk-tcpipstack_amd", "rxg", "librxg_exp.so"))
os.environ.setdefault("RXG_LIB_OVERRIDE", "1")  # the experiment library, on purpose (rxg.load_library)
import rxg  # noqa: E402

WL = {"c3": (1500, 1000, 0), "c2": (64, 1, 0), "c4": (0, 65536, 1)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workloads", default="c3,c4,c2")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--frames", type=int, default=1 << 20)
    ap.add_argument("--variants", default="0", help="RXG_PG_VARIANT values, interleaved")
    ap.add_argument("--check", action="store_true")
    args = ap.parse_args()
    engs = {}
    for v in args.variants.split(","):
        os.environ["RXG_PG_VARIANT"] = v
        engs[v] = rxg.Engine(0)
    eng = engs[args.variants.split(",")[0]]
    n = args.frames
    for w in args.workloads.split(","):
        L, flows, mix = WL[w]
        b = eng.synth(n=n, nflows=flows, len_a=L or 1500, mix=mix, seed=5)
        tcb, live = rxg.synthetic_tcb_table(flows)
        eng.tcb_load(tcb, live)
        recs = eng.alloc(n * 16)
        eng.rx_burst_dev(b["arena"].ptr, b["off64"].ptr, b["len"].ptr, n, recs.ptr, 16)
        lens = b["len"].download(np.uint16, n).astype(np.int64)
        pl = (lens - 54).clip(min=0)
        cap = int(((pl + 127) // 128 * 128).sum())  # room for every alignment variant
        arena, msgs, used = eng.alloc(cap), eng.alloc(n * 16), eng.alloc(8)
        res = {v: [] for v in engs}
        for rnd in range(3):
            for v, e2 in engs.items():
                e2.tcb_load(tcb, live)
                e2.rx_burst_dev(b["arena"].ptr, b["off64"].ptr, b["len"].ptr, n, recs.ptr, 16)
                for _ in range(2):
                    e2.payload_gather_dev(arena.ptr, cap, msgs.ptr, used.ptr)
                evs = [(e2.event(), e2.event()) for _ in range(args.iters)]
                for a, e in evs:
                    e2.record(a)
                    e2.payload_gather_dev(arena.ptr, cap, msgs.ptr, used.ptr)
                    e2.record(e)
                e2.sync()
                res[v] += [e2.elapsed_ms(a, e) for a, e in evs]
        if args.check:
            ref = None
            for v, e2 in engs.items():
                e2.payload_gather_dev(arena.ptr, cap, msgs.ptr, used.ptr)
                e2.sync()
                m = msgs.download(np.uint64, 2 * n).reshape(n, 2)
                ar = arena.download(np.uint8, cap)
                offs, ln = m[:, 0].astype(np.int64), (m[:, 1] & 0xFFFFFFFF).astype(np.int64)
                u = int(used.download(np.uint64, 1)[0])
                body = np.concatenate([ar[o:o + l] for o, l in zip(offs[:4096], ln[:4096])])
                gaps = [ar[o + l:nxt] for o, l, nxt in zip(offs[:4095], ln[:4095], offs[1:4096]) if l]
                zero = all((g == 0).all() for g in gaps)
                if ref is None:
                    ref = body
                print(json.dumps({"variant": v, "workload": w, "used": u, "same_payload": bool(np.array_equal(body, ref)),
                                  "pad_zero": bool(zero), "align": int(np.gcd.reduce(offs[ln > 0][:4096]))}), flush=True)
        alg = 2 * int(pl.sum()) + 32 * n
        for v, ms in res.items():
            ms = np.array(ms)
            k = float(np.median(ms)) / 1e3
            print(json.dumps({"variant": v, "workload": w, "us_median": round(k * 1e6, 2),
                              "us_min": round(ms.min() * 1e3, 2), "alg_bytes": alg,
                              "GBps": round(alg / k / 1e9, 1), "frac_8TBs": round(alg / k / 8e12, 4)}),
                  flush=True)
        for d in (recs, arena, msgs, used):
            d.free()
        for v in b.values():
            if isinstance(v, rxg.DevArray):
                v.free()


if __name__ == "__main__":
    main()
