#!/usr/bin/env python3
"""A fixed number of rx launches of one bench workload through the product library, for
rocprofv3 (kernel trace / PMC passes): scripts/gpu_prof.sh.  The same synthetic batches,
tables and launch forms as bench.py; no timing of its own.
  python scripts/profrun.py --workload c2multi --iters 20 [--rec 8] [--prov build.json]

--prov writes rxg.build_provenance() of the library this process loaded (its src= hash) to a
file: scripts/gpu_prof.sh stamps every traffic.json and kernel-trace directory with it."""
import json
import argparse
import os
import sys

import torch  # noqa: F401  (one HIP runtime per process)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dpdk-tcpipstack_amd")]
import rxg  # noqa: E402

# name: (frame_len, flows, mix, rotating copies) -- bench.py WORKLOADS
WL = {"c3": (1500, 1000, 0, 2), "c2": (64, 1, 0, 16), "c4": (0, 65536, 1, 3)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="c3", choices=sorted(WL) + ["c2s", "c2multi", "c2multis", "tx3", "tx4", "pg3", "pg4",
                                                                      "pf3", "pf4", "pr3", "pr4"])
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--frames", type=int, default=1 << 20)
    ap.add_argument("--rec", type=int, default=16, choices=[8, 16, 48])
    ap.add_argument("--prov", default=None, help="write the loaded library's build provenance here")
    args = ap.parse_args()
    rec = args.rec
    eng = rxg.Engine(0)
    if args.prov:
        with open(args.prov, "w") as fh:
            json.dump(rxg.build_provenance(), fh, indent=1)
    n = args.frames
    if args.workload in ("c2multi", "c2multis"):  # bench.py multiburst_leg: 16 bursts of one 1 GiB pool per launch
        k = 16
        pool = eng.synth(n=n * k, nflows=1, len_a=64, mix=0, seed=0x5EED0001 + 123)
        eng.tcb_load(*rxg.synthetic_tcb_table(1))
        out = eng.alloc(n * k * rec)
        if args.workload == "c2multis":  # the fixed-stride form: frame i of burst j at slot j n + i
            sb = [(j * n, pool["len"].ptr + j * n * 2, n, out.ptr + j * n * rec) for j in range(k)]
            for _ in range(args.iters):
                eng.rx_bursts_strided_dev(pool["arena"].ptr, 1, sb, rec)
            eng.sync()
            return
        bursts = [(pool["off64"].ptr + j * n * 4, pool["len"].ptr + j * n * 2, n, out.ptr + j * n * rec)
                  for j in range(k)]
        for _ in range(args.iters):
            eng.rx_bursts_dev(pool["arena"].ptr, bursts, rec)
        eng.sync()
        return
    if args.workload[:2] in ("pf", "pr"):
        # bench.py fused_leg: rxg_rx_burst_payload_dev over the C3 / C4 batches (rotating copies),
        # each with a payload arena of the pool's size ("pr": by reference, no arena)
        L, flows, mix, copies = WL["c3" if args.workload[2] == "3" else "c4"]
        bs = [eng.synth(n=n, nflows=flows, len_a=L or 1500, mix=mix, seed=0x5EED0001 + 17 * c) for c in range(copies)]
        eng.tcb_load(*rxg.synthetic_tcb_table(flows))
        out, msgs = eng.alloc(n * rec), eng.alloc(n * 16)
        arenas = [eng.alloc(b["arena_bytes"]) for b in bs] if args.workload[:2] == "pf" else None
        for i in range(args.iters):
            b = bs[i % copies]
            eng.rx_burst_payload_dev(b["arena"].ptr, b["off64"].ptr, b["len"].ptr, n, out.ptr,
                                     arenas[i % copies].ptr if arenas else 0, msgs.ptr, rec)
        eng.sync()
        return
    if args.workload[:2] in ("tx", "pg"):
        # bench.py tx_leg / payload_leg over the C3 ("3") or C4 ("4") batch: rxg_tx_cksum_dev
        # in place (the batch's checksums are already the generated ones), or one rx burst then
        # rxg_payload_gather_dev into an arena of exactly the burst's size
        L, flows, mix, copies = WL["c3" if args.workload[2] == "3" else "c4"]
        b = eng.synth(n=n, nflows=flows, len_a=L or 1500, mix=mix, seed=0x5EED0001)
        eng.tcb_load(*rxg.synthetic_tcb_table(flows))
        if args.workload[:2] == "tx":
            for _ in range(args.iters):
                eng.tx_cksum_dev(b["arena"].ptr, b["off64"].ptr, b["len"].ptr, n)
            eng.sync()
            return
        import numpy as np
        out = eng.alloc(n * rec)
        eng.rx_burst_dev(b["arena"].ptr, b["off64"].ptr, b["len"].ptr, n, out.ptr, rec)
        pl = (b["len"].download(np.uint16, n).astype(np.int64) - 54).clip(min=0)
        cap = int(((pl + 15) // 16 * 16).sum())
        arena, msgs, used = eng.alloc(cap), eng.alloc(n * 16), eng.alloc(8)
        for _ in range(args.iters):
            eng.payload_gather_dev(arena.ptr, cap, msgs.ptr, used.ptr)
        eng.sync()
        assert int(used.download(np.uint64, 1)[0]) == cap
        return
    strided = args.workload == "c2s"  # C2 through rxg_rx_bursts_strided_dev (frame i at slot i)
    L, flows, mix, copies = WL["c2" if strided else args.workload]
    bs = [eng.synth(n=n, nflows=flows, len_a=L or 1500, mix=mix, seed=0x5EED0001 + 17 * c) for c in range(copies)]
    eng.tcb_load(*rxg.synthetic_tcb_table(flows))
    out = eng.alloc(n * rec)
    for i in range(args.iters):
        b = bs[i % copies]
        if strided:
            eng.rx_bursts_strided_dev(b["arena"].ptr, 1, [(0, b["len"].ptr, n, out.ptr)], rec)
        else:
            eng.rx_burst_dev(b["arena"].ptr, b["off64"].ptr, b["len"].ptr, n, out.ptr, rec)
    eng.sync()


if __name__ == "__main__":
    main()
