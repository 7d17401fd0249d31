#!/usr/bin/env python3
"""A/B of the fused rx + payload hand-off (rxg_rx_burst_payload_dev) in one process, through
the experiment library: RXG_VARIANT 0 = production; round 5's forms 101-107 (plain /
chunk-granular / pipelined / 4-waves stores) were measured with it and removed again
(profiles/r05/fused/).  A variant "V@G" caps the grid at G workgroups.  Per workload (C3
1500 B / 1 K flows, C4 IMIX / 64 K flows, C2 64 B / 1 flow; 2^20 frames, rotating batches as
bench.py), the mean kernel time over K launches (one event pair around them), interleaved
rounds, and a check that every variant writes the first one's records and messages; --shifts
places the payload arena at other offsets from the pool.  One JSON line per measurement.
  python scripts/fusedbench.py [--variants 0,0@512] [--rounds 3] [--steps 20] [--copy-ref] [--by-ref]"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dpdk-tcpipstack_amd")]
os.environ.setdefault("RXG_LIB", os.path.join(ROOT, "dpdk-tcpipstack_amd", "rxg", "librxg_exp.so"))
os.environ.setdefault("RXG_LIB_OVERRIDE", "1")  # the experiment library, on purpose (rxg.load_library)
import numpy as np  # noqa: E402
import torch  # noqa: E402,F401

import rxg  # noqa: E402

WL = {"c3": (1500, 1000, 0, 2), "c4": (0, 65536, 1, 3), "c2": (64, 1, 0, 16)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", default="0", help="forms (RXG_VARIANT), each optionally @grid")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--workloads", default="c3,c4,c2")
    ap.add_argument("--rec", type=int, default=8)
    ap.add_argument("--shifts", default="0", help="payload arena base offsets to try (bytes, multiples of 64)")
    ap.add_argument("--copy-ref", action="store_true", help="also time a device-to-device copy of 1.5 GiB")
    ap.add_argument("--by-ref", action="store_true", help="the by-reference form (payload arena NULL: messages only)")
    args = ap.parse_args()
    # a variant "V@G" runs form V on a grid capped at G workgroups (rxg_config.max_blocks)
    variants = args.variants.split(",")
    engines = {}
    for v in variants:
        form, _, grid = v.partition("@")
        os.environ["RXG_VARIANT"] = form
        engines[v] = rxg.Engine(0, max_blocks=int(grid or 0))
    os.environ["RXG_VARIANT"] = "0"
    n, rec = 1 << 20, args.rec
    e0 = engines[variants[0]]
    for w in args.workloads.split(","):
        L, flows, mix, copies = WL[w]
        bs = [e0.synth(n=n, nflows=flows, len_a=L or 1500, mix=mix, seed=0x5EED0001 + 17 * c) for c in range(copies)]
        e0.sync()
        tcb, live = rxg.synthetic_tcb_table(flows)
        for e in engines.values():
            e.tcb_load(tcb, live)
            e.tcb_sync()
        shifts = [int(x) for x in args.shifts.split(",")]
        arenas = [e0.alloc(b["arena_bytes"] + max(shifts)) for b in bs]
        out, msgs = e0.alloc(n * rec), e0.alloc(n * 16)
        ref = None
        for r in range(args.rounds):
            for v, sh in [(v, sh) for v in variants for sh in shifts]:
                e = engines[v]

                def launch(i):
                    b = bs[i % copies]
                    e.rx_burst_payload_dev(b["arena"].ptr, b["off64"].ptr, b["len"].ptr, n, out.ptr,
                                           0 if args.by_ref else arenas[i % copies].ptr + sh, msgs.ptr, rec)
                for i in range(3):
                    launch(i)
                e.sync()
                ev0, ev1 = e.event(), e.event()
                e.record(ev0)
                for i in range(args.steps):
                    launch(i)
                e.record(ev1)
                e.sync()
                us = e.elapsed_ms(ev0, ev1) / args.steps * 1e3
                e.event_destroy(ev0)
                e.event_destroy(ev1)
                # the last launch's batch: records, messages and the written payload lines
                got = (out.download(np.uint8, n * rec).tobytes(), msgs.download(np.uint8, n * 16).tobytes(),
                       arenas[(args.steps - 1) % copies].download(np.uint8, 1 << 22).tobytes())
                if ref is None:
                    ref = got
                same = got[:2] == ref[:2]
                delta = (arenas[0].ptr + sh) - bs[0]["arena"].ptr
                print(json.dumps({"round": r, "workload": w, "variant": v, "by_ref": args.by_ref, "arena_shift": sh,
                                  "arena_minus_pool": delta, "kernel_us": round(us, 2),
                                  "same_records_and_msgs": bool(same)}), flush=True)
        for d in arenas + [out, msgs]:
            d.free()
        for b in bs:
            for x in b.values():
                if isinstance(x, rxg.DevArray):
                    x.free()
    if args.copy_ref:
        # the box's device-to-device copy rate for the same bytes (torch's copy kernel): the
        # fused C3 launch reads the frames and writes about as many payload-line bytes
        nbytes = (1 << 20) * 1536
        src = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
        dst = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
        for r in range(args.rounds):
            for _ in range(3):
                dst.copy_(src)
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for _ in range(args.steps):
                dst.copy_(src)
            b.record()
            torch.cuda.synchronize()
            us = a.elapsed_time(b) / args.steps * 1e3
            print(json.dumps({"round": r, "workload": "copy_1536MiB_d2d", "kernel_us": round(us, 2),
                              "moved_TBps": round(2 * nbytes / us / 1e6, 3)}), flush=True)
    for e in engines.values():
        e.close()


if __name__ == "__main__":
    main()
