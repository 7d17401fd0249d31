#!/usr/bin/env python3
"""The faithful oracle (bench.py's cpu_baseline "port") timed on the shape SURVEY.md §6 timed
the reference's own hot-path files on: 1 500 B frames, 1 000 flows from 1 000 source IPs, +verify,
after one pass has taught the ARP list every source.  Run in the survey's container class (no
GPU needed), it gives the port / reference factor bench.py states beside its CPU baseline
(HISTORY.md §6.R5).  Prints one JSON line.
  python scripts/cpu_calib.py [--seconds 5] [--frames 20000]"""
import argparse
import json
import os
import platform
import random
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "dpdk-tcpipstack_amd")]
import oracle  # noqa: E402
import pktgen  # noqa: E402
import rxg  # noqa: E402

SURVEY_REFERENCE_MPPS = {"O0": 0.0121, "O2": 0.0185}  # SURVEY.md §6, same shape, the reference's files


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=5.0)
    ap.add_argument("--frames", type=int, default=20000)
    args = ap.parse_args()
    flows = 1000
    rng = random.Random(0x5EED0002)
    frames = []
    for i in range(args.frames):
        f = i if i < flows else rng.randrange(flows)  # every source once, then uniform
        src = pktgen.ip4(10, (f >> 16) & 255, (f >> 8) & 255, f & 255)
        frames.append(pktgen.frame(src_ip=src, sport=1024 + f, payload=rng.randbytes(1446),
                                   src_mac=bytes([2, 0, 10, (f >> 16) & 255, (f >> 8) & 255, f & 255])))
    arena, off, lens = pktgen.pack_arena(frames)
    tcb, live = rxg.synthetic_tcb_table(flows)
    out = {"shape": "1500 B, 1000 flows / 1000 src IPs, +verify", "frames": args.frames,
           "cpu": platform.processor() or platform.machine()}
    for opt in ("O0", "O2"):
        oracle.arp_reset()
        rec, _ = oracle.rx_batch(arena, off, lens, tcb, live, faithful=True, opt=opt)  # learn ARP
        assert (rec["c"]["verdict"] == 0).all() and oracle.lib(opt).orc_arp_count() == flows
        pk, s, t0 = 0, 0, time.perf_counter()
        while time.perf_counter() - t0 < args.seconds:
            e = min(s + 2000, len(frames))
            oracle.rx_batch(arena, off[s:e], lens[s:e], tcb, live, faithful=True, opt=opt)
            pk += e - s
            s = 0 if e >= len(frames) else e
        mpps = pk / (time.perf_counter() - t0) / 1e6
        out[f"port_mpps_{opt}"] = round(mpps, 6)
        out[f"reference_over_port_{opt}"] = round(SURVEY_REFERENCE_MPPS[opt] / mpps, 3)
    oracle.arp_reset()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
