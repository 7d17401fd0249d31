#!/usr/bin/env python3
"""Kernel micro-benchmark: interleaved rounds of kernel variants in ONE process
(cdna_hip_programming.md §5.4 rule 24).  Variants are (RXG_VARIANT, RXG_MAX_BLOCKS) pairs;
each gets its own rxg context; all share the same device-resident workloads.

  python scripts/kbench.py --variants 0:2048,2:2048 --workloads c3,c2 --rounds 5
"""
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

WL = {"c3": (1500, 1000, 0, 2), "c3r1": (1500, 1000, 0, 1), "c4r4": (0, 65536, 1, 4), "c2": (64, 1, 0, 16), "c4": (0, 65536, 1, 3),
      "c2r1": (64, 1, 0, 1), "c2x4": (64, 1, 0, 4),
      # single-size legs of the IMIX (64 K flows): where C4's time goes
      "u64": (64, 65536, 0, 16), "u576": (576, 65536, 0, 2), "u1500": (1500, 65536, 0, 1),
      # C4's IMIX at other flow counts (the TCB table's size: 16 K flows 1 MiB ... 256 K 16 MiB)
      "c4f1k": (0, 1024, 1, 3), "c4f16k": (0, 16384, 1, 3), "c4f256k": (0, 262144, 1, 3),
      # C2 as 16 bursts of one 1 GiB pool per launch (rxg_rx_bursts_dev, bench.py multiburst_leg)
      "c2m": (64, 1, 0, 1)}
MULTI = 16


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", default="0:2048")
    ap.add_argument("--workloads", default="c3,c2")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--frames", type=int, default=1 << 20)
    ap.add_argument("--frames-c2", type=int, default=0, help="override frames for c2* workloads")
    ap.add_argument("--rec", type=int, default=16)
    ap.add_argument("--seed", type=int, default=77, help="copy c is synthesised with seed + c * seed_step")
    ap.add_argument("--seed-step", type=int, default=1, help="17 with bench.py's seed reproduces its batches")
    ap.add_argument("--tx", action="store_true", help="time rxg_tx_cksum_dev (rx_kernel<0>) instead")
    ap.add_argument("--stream", action="store_true",
                    help="launch and time on a caller stream (a torch stream), not the context's own: "
                         "the table-reader ordering of DESIGN.md §2.4 runs per launch")
    ap.add_argument("--engine-flags", type=int, default=0,
                    help="rxg_config.flags of every variant's context (2 = RXG_CFG_STREAMS_OUTLIVE_WRITES)")
    ap.add_argument("--check", action="store_true",
                    help="also compare every variant's records (and counters) with the first variant's")
    args = ap.parse_args()

    base = rxg.Engine(0)
    st = torch.cuda.Stream(device=0).cuda_stream if args.stream else None
    wls = {}
    for w in args.workloads.split(","):
        L, flows, mix, copies = WL[w]
        nfr = args.frames_c2 if (w.startswith("c2") and args.frames_c2) else args.frames
        if w == "c2m":  # one pool of MULTI bursts; the workload's bytes are the whole launch's
            pool = base.synth(n=nfr * MULTI, nflows=1, len_a=64, mix=0, seed=77)
            tcb, live = rxg.synthetic_tcb_table(1)
            wls[w] = ([pool], nfr * MULTI * 64, tcb, live, nfr)
            continue
        bs = [base.synth(n=nfr, nflows=flows, len_a=L or 1500, mix=mix, seed=args.seed + c * args.seed_step)
              for c in range(copies)]
        lens = bs[0]["len"].download(np.uint16, nfr)
        tcb, live = rxg.synthetic_tcb_table(flows)
        wls[w] = (bs, int(lens.astype(np.uint64).sum()), tcb, live, nfr)
    nout = max(args.frames, args.frames_c2) * (MULTI if "c2m" in wls else 1)
    out = base.alloc(nout * args.rec)
    base.sync()

    # A variant may name another build of librxg (4th field, a path): A/B of two builds in
    # one process.  The binding's module-level library handle is switched per engine.
    main_lib = rxg.load_library()
    libs, engines, arp_on = {}, {}, {}
    for v in args.variants.split(","):
        parts = v.split(":")
        os.environ["RXG_VARIANT"] = parts[0]
        os.environ["RXG_MAX_BLOCKS"] = parts[1]
        os.environ["RXG_NOCOUNT"] = "1" if (len(parts) > 2 and parts[2] == "nc") else "0"
        # 5th field: the mirror's load limit in percent (RXG_MIRROR_LOAD_PCT)
        os.environ["RXG_MIRROR_LOAD_PCT"] = parts[4] if len(parts) > 4 and parts[4] else "50"
        lib = main_lib
        if len(parts) > 3 and parts[3]:
            rxg._lib = None
            lib = rxg.load_library(parts[3])
        rxg._lib = lib
        libs[v] = lib
        # 6th field "arp": the ARP mirror on, loaded with every flow's source (ip.c:30-32 finds
        # them all: the kernel's ARP probe runs, RXG_F_ARP_LEARN stays clear)
        arp_on[v] = len(parts) > 5 and parts[5] == "arp"
        engines[v] = rxg.Engine(0, flags=args.engine_flags)
        if st is not None and hasattr(lib, "rxg_stream_register"):  # (older builds: no such call)
            engines[v].stream_register(st)  # needed by RXG_CFG_STREAMS_OUTLIVE_WRITES contexts
        rxg._lib = main_lib
    res = {(v, w): [] for v in engines for w in wls}
    for r in range(args.rounds):
        for w, (bs, nbytes, tcb, live, nfr) in wls.items():
            for v, eng in engines.items():
                rxg._lib = libs[v]
                eng.tcb_load(tcb, live)
                if arp_on[v]:
                    eng.arp_load(tcb["ipv4_src"][1:])
                eng.tcb_sync()
                evs = [(eng.event(), eng.event()) for _ in range(args.iters)]
                def launch(b):
                    if w == "c2m":
                        R = args.rec
                        eng.rx_bursts_dev(b["arena"].ptr, [(b["off64"].ptr + j * nfr * 4, b["len"].ptr + j * nfr * 2,
                                                            nfr, out.ptr + j * nfr * R) for j in range(MULTI)], R)
                    elif args.tx:  # the batch's checksums are already right: rewriting keeps them
                        eng.tx_cksum_dev(b["arena"].ptr, b["off64"].ptr, b["len"].ptr, nfr)
                    else:
                        eng.rx_burst_dev(b["arena"].ptr, b["off64"].ptr, b["len"].ptr, nfr, out.ptr, args.rec, st)
                for i in range(2):
                    launch(bs[i % len(bs)])
                for i in range(args.iters):
                    b = bs[(i + 2) % len(bs)]
                    eng.record(evs[i][0], st)
                    launch(b)
                    eng.record(evs[i][1], st)
                eng.sync()
                if st is not None:
                    torch.cuda.synchronize(0)
                ms = [eng.elapsed_ms(a, b) for a, b in evs]
                res[(v, w)].append(ms)
                for a, b in evs:
                    libs[v].rxg_event_destroy(eng.ctx, a)
                    libs[v].rxg_event_destroy(eng.ctx, b)
                rxg._lib = main_lib
    if args.check and args.tx:
        # every variant regenerates the checksums of a copy of batch 0 whose four checksum
        # bytes were zeroed; the result must equal the synthesised batch byte for byte
        for w, (bs, nbytes, tcb, live, nfr) in wls.items():
            b = bs[0]
            ref = b["arena"].download(np.uint8, b["arena_bytes"])
            offs = b["off64"].download(np.uint32, nfr).astype(np.int64) * 64
            lens = b["len"].download(np.uint16, nfr).astype(np.int64)
            z = ref.copy()
            for bp in (24, 25, 50, 51):
                m = lens > bp
                z[offs[m] + bp] = 0
            for v, eng in engines.items():
                rxg._lib = libs[v]
                d = eng.to_device(z)
                eng.tx_cksum_dev(d.ptr, b["off64"].ptr, b["len"].ptr, nfr)
                eng.sync()
                got = d.download(np.uint8, b["arena_bytes"])
                d.free()
                rxg._lib = main_lib
                print(json.dumps({"check": w, "variant": v, "tx_bytes_equal": bool(np.array_equal(got, ref)),
                                  "zeroed_differs": bool(not np.array_equal(z, ref))}), flush=True)
    if args.check and not args.tx:
        for w, (bs, nbytes, tcb, live, nfr) in wls.items():
            ref = None
            for v, eng in engines.items():
                rxg._lib = libs[v]
                eng.tcb_load(tcb, live)
                if arp_on[v]:
                    eng.arp_load(tcb["ipv4_src"][1:])
                eng.tcb_sync()
                eng.counters_reset()
                if w == "c2m":
                    b = bs[0]
                    eng.rx_bursts_dev(b["arena"].ptr, [(b["off64"].ptr + j * nfr * 4, b["len"].ptr + j * nfr * 2,
                                                        nfr, out.ptr + j * nfr * args.rec) for j in range(MULTI)], args.rec)
                    nrec = nfr * MULTI
                else:
                    eng.rx_burst_dev(bs[0]["arena"].ptr, bs[0]["off64"].ptr, bs[0]["len"].ptr, nfr, out.ptr, args.rec)
                    nrec = nfr
                eng.sync()
                got = (out.download(np.uint8, nrec * args.rec).tobytes(), tuple(eng.counters()))
                rxg._lib = main_lib
                if ref is None:
                    ref = got
                print(json.dumps({"check": w, "variant": v, "records_equal": got[0] == ref[0],
                                  "counters_equal": got[1] == ref[1]}), flush=True)
    for (v, w), ms in res.items():
        nbytes = wls[w][1]
        med = float(np.median([np.median(r) for r in ms]))  # median over rounds of each round's median
        allm = [x for r in ms for x in r]
        print(json.dumps({"variant": v, "workload": w, "kernel_us_median": round(med * 1e3, 2),
                          "kernel_us_min": round(min(np.median(r) for r in ms) * 1e3, 2),
                          "kernel_us_mean_all": round(float(np.mean(allm)) * 1e3, 2),
                          "kernel_us_max_all": round(max(allm) * 1e3, 2),
                          "GBps": round(nbytes / (med * 1e-3) / 1e9, 1),
                          "frac_8TBs": round(nbytes / (med * 1e-3) / 8e12, 4)}), flush=True)


if __name__ == "__main__":
    main()
