#!/usr/bin/env python3
"""Where does bench.py's C4 leg lose time against C4 measured alone?  Replays the bench's
sequence (headline C3 workload, its REC16 twin, the C2 leg, then C4) on one engine and times
the C4 workload after each stage with bench.py's own Workload / time_workload.

  python scripts/c4ctx.py [--steps 30]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT]
import bench  # noqa: E402
import rxg  # noqa: E402  (bench put the package on the path)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=5)
    args = ap.parse_args()
    eng = rxg.Engine(device=0)
    n = 1 << 20
    seed = bench.shard_seed(0x5EED0001, 0)

    def c4(stage, wl=None):
        own = wl is None
        if own:
            wl = bench.Workload(eng, "c4_imix_64Kflows", n, seed + 99, rxg.REC8)
        t, l = rxg.synthetic_tcb_table(wl.flows)
        eng.tcb_load(t, l)
        _, k = bench.time_workload(eng, wl, args.steps, args.warmup, None, None)
        k = sorted(k)
        print(json.dumps({"stage": stage, "c4_us_mean": round(sum(k) / len(k) * 1e3, 2),
                          "c4_us_median": round(k[len(k) // 2] * 1e3, 2)}), flush=True)
        if own:
            wl.free()

    c4("fresh")
    w3 = bench.Workload(eng, "c3_1500B_1Kflows", n, seed, rxg.REC8)
    t3, l3 = rxg.synthetic_tcb_table(w3.flows)
    eng.tcb_load(t3, l3)
    bench.time_workload(eng, w3, args.steps, args.warmup, None, None)
    c4("after C3 workload (kept)")
    ow = bench.Workload(eng, "c3_1500B_1Kflows", n, seed, rxg.REC16)
    bench.time_workload(eng, ow, args.steps, args.warmup, None, None)
    ow.free()
    c4("after REC16 twin (freed)")
    w2 = bench.Workload(eng, "c2_64B_1flow", n, seed + 99, rxg.REC8)
    t2, l2 = rxg.synthetic_tcb_table(w2.flows)
    eng.tcb_load(t2, l2)
    bench.time_workload(eng, w2, args.steps, args.warmup, None, None)
    w2.free()
    c4("after C2 leg (freed), as bench.py")
    w3.free()
    c4("C3 workload freed")


if __name__ == "__main__":
    main()
