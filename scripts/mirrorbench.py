#!/usr/bin/env python3
"""Cost of tcbs[] mirror writes against the table size.

For Ntcb = 1 001 / 65 537 / 1 048 577 (C3 / C4 / C5 tables): k writes (half tcp_listen
children appended at Ntcb, half remove_tcb of random flows), then rxg_tcb_sync and a stream
sync; host wall time per sync, per write, with the product library (O(1) device patches; round
1's full rebuild per sync was measured through the retired experiment library, HISTORY.md):
  python scripts/mirrorbench.py
Prints one JSON line per (Ntcb, k)."""
import json
import os
import random
import sys
import time

import numpy as np
import torch  # noqa: F401  (one HIP runtime per process)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dpdk-tcpipstack_amd")]
import rxg  # noqa: E402


def main():
    eng = rxg.Engine(0)
    mode = "patch"
    rng = random.Random(1)
    dst = rxg.ip_raw(192, 168, 78, 2)
    for nflows in (1000, 65536, 1 << 20):
        t, live = rxg.synthetic_tcb_table(nflows)
        eng.tcb_load(t, live)
        eng.tcb_sync()
        eng.sync()
        n = nflows + 1
        for k in (1, 32, 1024):
            reps = 100
            ts = []
            for _ in range(reps):
                t0 = time.perf_counter()
                for j in range(k):
                    if j & 1:
                        i = rng.randrange(1, n)
                        eng.tcb_remove(i)
                    else:
                        eng.tcb_upsert(n, 80, rng.randrange(1024, 65536), dst,
                                       rxg.ip_host(172, 16, rng.randrange(256), rng.randrange(256)), 3)
                        n += 1
                eng.tcb_sync()
                eng.sync()
                ts.append(time.perf_counter() - t0)
            # the same writes' Python/ctypes call cost alone (no sync): subtracted below
            t0 = time.perf_counter()
            for j in range(k):
                eng.tcb_count()
            call = (time.perf_counter() - t0) / k
            med = float(np.median(ts))
            print(json.dumps({"mode": mode, "ntcb": n, "writes_per_sync": k, "sync_us_median": round(med * 1e6, 1),
                              "us_per_write": round(med * 1e6 / k, 2),
                              "ctypes_call_us": round(call * 1e6, 2), "reps": reps}), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
