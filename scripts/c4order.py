#!/usr/bin/env python3
"""C4 (IMIX 64/576/1500 7:4:1, 64 K flows) sensitivity to the class mix inside a slice.
The same device arena is classified through permuted descriptor lists (the kernel reads
frames only through off64/len), so only the order of frames changes:
  orig      the synthetic order (every 64-frame slice mixes ~37/21/5 frames per class)
  sortW     frames stably sorted by length inside windows of W frames
Prints the median kernel time of each order, interleaved rounds in one process."""
import json
import os
import sys

import numpy as np
import torch  # noqa: F401

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dpdk-tcpipstack_amd")]
import rxg  # noqa: E402


def main():
    n = 1 << 20
    eng = rxg.Engine(0)
    tcb, live = rxg.synthetic_tcb_table(65536)
    eng.tcb_load(tcb, live)
    b = eng.synth(n=n, nflows=65536, mix=1, seed=77)
    eng.sync()
    off = b["off64"].download(np.uint32, n)
    lens = b["len"].download(np.uint16, n)
    nbytes = int(lens.astype(np.uint64).sum())
    orders = {"orig": np.arange(n)}
    for w in [int(x) for x in (sys.argv[1:] or ["768", "6144", str(n)])]:
        idx = np.arange(n)
        key = (idx // w) * 4096 + lens.astype(np.int64)
        orders[f"sort{w}"] = np.argsort(key, kind="stable")
    dev = {}
    for k, p in orders.items():
        dev[k] = (eng.to_device(np.ascontiguousarray(off[p])), eng.to_device(np.ascontiguousarray(lens[p])))
    out = eng.alloc(n * 8)
    res = {k: [] for k in orders}
    for r in range(5):
        for k, (do, dl) in dev.items():
            evs = [(eng.event(), eng.event()) for _ in range(10)]
            for _ in range(2):
                eng.rx_burst_dev(b["arena"].ptr, do.ptr, dl.ptr, n, out.ptr, rxg.REC8)
            for a, e in evs:
                eng.record(a)
                eng.rx_burst_dev(b["arena"].ptr, do.ptr, dl.ptr, n, out.ptr, rxg.REC8)
                eng.record(e)
            eng.sync()
            res[k].append(float(np.median([eng.elapsed_ms(a, e) for a, e in evs])))
    cnt = eng.counters()
    for k, ms in res.items():
        med = float(np.median(ms))
        print(json.dumps({"order": k, "kernel_us": round(med * 1e3, 2),
                          "frac_8TBs": round(nbytes / (med * 1e-3) / 8e12, 4)}), flush=True)
    print(json.dumps({"tcp_cksum_bad": int(cnt[8])}))


if __name__ == "__main__":
    main()
