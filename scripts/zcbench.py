#!/usr/bin/env python3
"""Host-resident batches: copy-in (pinned H2D of arena + descriptors, kernel, D2H of the
records, one stream) vs zero-copy (the kernel reads the frames, descriptors and writes the
records straight from/to pinned host memory over PCIe: rxg_rx_burst_dev on host
pointers).  Also tx generate in place on host frames.  Prints GB/s and Mpps per case.
  python scripts/zcbench.py [workloads]"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dpdk-tcpipstack_amd")]
import torch  # noqa: E402,F401
import rxg  # noqa: E402

WL = {"c3": (1500, 1000, 0), "c4": (0, 65536, 1), "c2": (64, 1, 0)}


def timed(eng, fn, iters=10):
    fn()
    eng.sync()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    eng.sync()
    return (time.perf_counter() - t0) / iters


def c5(eng, n):
    """C5 shapes: tx (IMIX, generate in place) + rx (IMIX, classify) per step, 2^20 each."""
    flows = 1 << 20
    tcb, live = rxg.synthetic_tcb_table(flows)
    eng.tcb_load(tcb, live)
    tx = eng.synth(n=n, nflows=flows, mix=1, seed=11)
    rx = eng.synth(n=n, nflows=flows, mix=1, seed=12)
    eng.sync()
    h = {}
    for k, b in (("tx", tx), ("rx", rx)):
        h[k] = (eng.pinned(b["arena_bytes"]), eng.pinned(n * 4), eng.pinned(n * 2))
        eng.d2h(h[k][0].ptr, b["arena"].ptr, b["arena_bytes"])
        eng.d2h(h[k][1].ptr, b["off64"].ptr, n * 4)
        eng.d2h(h[k][2].ptr, b["len"].ptr, n * 2)
    hr = eng.pinned(n * 16)
    out = eng.alloc(n * 16)
    eng.sync()
    s2 = torch.cuda.Stream(device=0).cuda_stream

    def tx_copy(st):
        a, o, l = h["tx"]
        eng.h2d(tx["arena"].ptr, a.ptr, tx["arena_bytes"], st)
        eng.h2d(tx["off64"].ptr, o.ptr, n * 4, st)
        eng.h2d(tx["len"].ptr, l.ptr, n * 2, st)
        eng.tx_cksum_dev(tx["arena"].ptr, tx["off64"].ptr, tx["len"].ptr, n, st)
        eng.d2h(a.ptr, tx["arena"].ptr, tx["arena_bytes"], st)

    def tx_zc(st):
        a, o, l = h["tx"]
        eng.tx_cksum_dev(a.ptr, o.ptr, l.ptr, n, st)

    def rx_copy(st):
        a, o, l = h["rx"]
        eng.h2d(rx["arena"].ptr, a.ptr, rx["arena_bytes"], st)
        eng.h2d(rx["off64"].ptr, o.ptr, n * 4, st)
        eng.h2d(rx["len"].ptr, l.ptr, n * 2, st)
        eng.rx_burst_dev(rx["arena"].ptr, rx["off64"].ptr, rx["len"].ptr, n, out.ptr, 16, st)
        eng.d2h(hr.ptr, out.ptr, n * 16, st)

    def rx_zc(st):
        a, o, l = h["rx"]
        eng.rx_burst_dev(a.ptr, o.ptr, l.ptr, n, hr.ptr, 16, st)

    def both_sync():
        eng.sync()
        eng.stream_sync(s2)

    cases = {"copy_1stream": lambda: (tx_copy(None), rx_copy(None)),
             "copy_2streams": lambda: (tx_copy(s2), rx_copy(None)),
             "txzc_rxcopy_2streams": lambda: (tx_zc(s2), rx_copy(None)),
             "zc_1stream": lambda: (tx_zc(None), rx_zc(None)),
             "zc_2streams": lambda: (tx_zc(s2), rx_zc(None))}
    for name, fn in cases.items():
        fn()
        both_sync()
        t0 = time.perf_counter()
        for _ in range(8):
            fn()
        both_sync()
        dt = (time.perf_counter() - t0) / 8
        print(json.dumps({"workload": "c5", "case": name, "ms": round(dt * 1e3, 3),
                          "mpps_per_direction": round(n / dt / 1e6, 2)}), flush=True)


def main():
    eng = rxg.Engine(0)
    n = 1 << 20
    if sys.argv[1:] == ["c5"]:
        c5(eng, n)
        return
    for w in (sys.argv[1:] or ["c3", "c4"]):
        L, flows, mix = WL[w]
        b = eng.synth(n=n, nflows=flows, len_a=L or 1500, mix=mix, seed=3)
        eng.sync()
        tcb, live = rxg.synthetic_tcb_table(flows)
        eng.tcb_load(tcb, live)
        nb = b["arena_bytes"]
        nbytes = int(b["len"].download(np.uint16, n).astype(np.int64).sum())
        ha, ho, hl, hr = eng.pinned(nb), eng.pinned(n * 4), eng.pinned(n * 2), eng.pinned(n * 16)
        eng.d2h(ha.ptr, b["arena"].ptr, nb)
        eng.d2h(ho.ptr, b["off64"].ptr, n * 4)
        eng.d2h(hl.ptr, b["len"].ptr, n * 2)
        out = eng.alloc(n * 16)
        eng.sync()

        def copy_in():
            eng.h2d(b["arena"].ptr, ha.ptr, nb)
            eng.h2d(b["off64"].ptr, ho.ptr, n * 4)
            eng.h2d(b["len"].ptr, hl.ptr, n * 2)
            eng.rx_burst_dev(b["arena"].ptr, b["off64"].ptr, b["len"].ptr, n, out.ptr, 16)
            eng.d2h(hr.ptr, out.ptr, n * 16)

        def zero_copy():
            eng.rx_burst_dev(ha.ptr, ho.ptr, hl.ptr, n, hr.ptr, 16)

        def tx_zero_copy():
            eng.tx_cksum_dev(ha.ptr, ho.ptr, hl.ptr, n)

        eng.counters_reset()
        for name, fn in (("rx_copy_in", copy_in), ("rx_zero_copy", zero_copy), ("tx_zero_copy", tx_zero_copy)):
            dt = timed(eng, fn)
            print(json.dumps({"workload": w, "case": name, "ms": round(dt * 1e3, 3),
                              "mpps": round(n / dt / 1e6, 2), "GBps": round(nbytes / dt / 1e9, 2)}), flush=True)
        rec = hr.np[: n * 16].view(rxg.REC16_DTYPE)
        c = eng.counters()
        print(json.dumps({"workload": w, "records_ok": bool((rec["verdict"] == 0).all() and (rec["tcp_cksum"] == 0).all()),
                          "tcp_cksum_bad": int(c[8])}), flush=True)
        for a in (ha, ho, hl, hr):
            a.free()
        out.free()
        for v in b.values():
            if isinstance(v, rxg.DevArray):
                v.free()
    eng.close()


if __name__ == "__main__":
    main()
