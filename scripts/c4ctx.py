#!/usr/bin/env python3
"""Where does bench.py's C4 leg lose time against C4 measured alone?  Replays the bench's
sequence (headline C3 workload, its REC16 twin, the C2 leg, then C4) on one engine and times
the C4 workload after each stage with bench.py's own Workload / time_workload.  Stages marked
"kept" re-time the batches allocated first (same buffers), so a placement effect (where the
allocation lands) separates from a state effect (what ran before).

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

    def c4(stage, wl=None, e=None):
        e = e or eng
        own = wl is None
        if own:
            wl = bench.Workload(e, "c4_imix_64Kflows", n, seed + 99, rxg.REC8)
        t, l = rxg.synthetic_tcb_table(wl.flows)
        e.tcb_load(t, l)
        _, k = bench.time_workload(e, wl, args.steps, args.warmup, None, None)
        k = sorted(k)
        print(json.dumps({"stage": stage, "c4_us_mean": round(sum(k) / len(k) * 1e3, 2),
                          "c4_us_median": round(k[len(k) // 2] * 1e3, 2)}), flush=True)
        if own:
            wl.free()

    first = bench.Workload(eng, "c4_imix_64Kflows", n, seed + 99, rxg.REC8)
    c4("fresh (kept batches)", first)
    c4("fresh, new batches")
    w3 = bench.Workload(eng, "c3_1500B_1Kflows", n, seed, rxg.REC8)
    t3, l3 = rxg.synthetic_tcb_table(w3.flows)
    eng.tcb_load(t3, l3)
    bench.time_workload(eng, w3, args.steps, args.warmup, None, None)
    c4("after C3 workload: kept batches", first)
    c4("after C3 workload: new batches")
    e2 = rxg.Engine(device=0)
    c4("after C3 workload: new engine, kept batches", first, e2)
    c4("after C3 workload: new engine, new batches", None, e2)
    e2.close()
    w3.free()
    c4("C3 freed: kept batches", first)
    c4("C3 freed: new batches")
    first.free()


if __name__ == "__main__":
    main()
