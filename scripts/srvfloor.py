#!/usr/bin/env python3
"""Where a served burst's microseconds go: the latency-mode server of the
experiment library with parts removed (timing only; records are not checked):
  RXG_VARIANT 0  production          79  no rx body (mailbox, acquire, release, done)
              80 no acquire at the request   81  no release before done   82  neither
Prints one JSON line: device-resident bursts of 1 and 32 frames (rxg_server_burst_dev) and
host bursts of 32 x 64 B (rxg_rx_burst, device staging), median us per call.

  for v in 0 79 80 81 82; do RXG_LIB=dpdk-tcpipstack_amd/rxg/librxg_exp.so RXG_VARIANT=$v \
      python scripts/srvfloor.py; done"""
import ctypes as C
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dpdk-tcpipstack_amd")]
import torch  # noqa: E402,F401
import rxg  # noqa: E402


def per_call_us(fn, budget=0.3):
    for _ in range(20):
        fn()
    lat, t0 = [], time.perf_counter()
    while time.perf_counter() - t0 < budget or len(lat) < 50:
        a = time.perf_counter()
        fn()
        lat.append(time.perf_counter() - a)
    return round(float(np.median(lat)) * 1e6, 2)


def main():
    n = 256
    eng = rxg.Engine(0, max_batch=n, max_bytes=n * 1536)
    lib = rxg.load_library()
    b = eng.synth(n=n, nflows=1000, len_a=64, seed=5)
    eng.sync()
    off = b["off64"].download(np.uint32, n)
    lens = b["len"].download(np.uint16, n)
    arena = b["arena"].download(np.uint8, b["arena_bytes"])
    tcb, live = rxg.synthetic_tcb_table(1000)
    eng.tcb_load(tcb, live)
    views = (rxg.PktView * n)(*[rxg.PktView(arena.ctypes.data + int(o) * 64, 0, int(ln), 0) for o, ln in zip(off, lens)])
    out = np.zeros(n, dtype=rxg.REC8_DTYPE)
    out_p = out.ctypes.data  # once: numpy's .ctypes.data costs ~2 us per access in Python
    d_out = eng.alloc(n * 8)
    eng.server_start(rxg.REC8, blocks=1, max_frames=n)
    row = {"variant": int(os.environ.get("RXG_VARIANT", "0")),
           "placement": {rxg.SRV_DEVICE: "device", rxg.SRV_HOST: "host"}[eng.server_placement()]}
    for k in (1, 32):
        dref = C.byref(rxg.DevBatch(b["arena"].ptr, b["off64"].ptr, b["len"].ptr, k, rxg.REC8, d_out.ptr))
        row[f"dev_{k}"] = per_call_us(lambda: lib.rxg_server_burst_dev(eng.ctx, dref))
    row["host_32x64B"] = per_call_us(lambda: lib.rxg_rx_burst(eng.ctx, views, 32, rxg.REC8, out_p))
    eng.server_stop()
    print(json.dumps(row), flush=True)
    d_out.free()
    eng.close()


if __name__ == "__main__":
    main()
