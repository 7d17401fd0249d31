#!/usr/bin/env python3
"""Working-set sweep for the C3 kernel: is the 1 GPU number helped by the 256 MiB
Infinity Cache or by warm address translations?  Times rx_burst_dev (REC16) over
  - 1 batch of 2^20 frames reused (bench.py's C3),
  - K separate batches of 2^20 frames in rotation (K x 1.5 GB),
  - 1 batch of K x 2^20 frames (one launch covers K x 1.5 GB).
Prints one JSON line per case with the mean kernel time per 2^20 frames."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dpdk-tcpipstack_amd")]
import torch  # noqa: E402,F401
import bench  # noqa: E402
import rxg  # noqa: E402


def run(eng, name, n, copies, steps=20, warmup=3):
    bench.WORKLOADS[name] = (1500, 1000, 0, copies)
    wl = bench.Workload(eng, name, n, 0x5EED0001, rxg.REC16)
    _, kern = bench.time_workload(eng, wl, steps, warmup, None, None)
    per_m = float(np.mean(kern)) * 1e3 * (1 << 20) / n
    gbs = wl.bytes_per_batch / (float(np.mean(kern)) / 1e3) / 1e9
    wl.free()
    print(json.dumps({"case": name, "frames_per_launch": n, "copies": copies,
                      "us_per_2^20_frames": round(per_m, 1), "GBps": round(gbs, 1)}), flush=True)


def main():
    eng = rxg.Engine(0)
    tcb, live = rxg.synthetic_tcb_table(1000)
    eng.tcb_load(tcb, live)
    ks = [int(k) for k in (sys.argv[1:] or ["1", "2", "4", "8"])]
    for k in ks:
        run(eng, f"rot{k}", 1 << 20, k)
    for k in ks[1:]:
        run(eng, f"big{k}", k << 20, 1)
    eng.close()


if __name__ == "__main__":
    main()
