#!/usr/bin/env python3
"""Debug: production (pieces) against experiment variant 52 (whole slices) on the C5 batch:
which frames differ after tx generate and after rx classify."""
import os
import sys

import numpy as np
import torch  # noqa: F401

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dpdk-tcpipstack_amd")]
os.environ.setdefault("RXG_LIB", os.path.join(ROOT, "dpdk-tcpipstack_amd", "rxg", "librxg_exp.so"))
import rxg  # noqa: E402

N = 1 << 20
engs = {}
for v in ("0", "52"):
    os.environ["RXG_VARIANT"] = v
    engs[v] = rxg.Engine(0)
mix = int(sys.argv[1]) if len(sys.argv) > 1 else 1
tcb, live = rxg.synthetic_tcb_table(N)
res = {}
for v, e in engs.items():
    b = e.synth(n=N, nflows=N, mix=mix, len_a=1500, seed=0xC5C5, with_flows=True)
    e.sync()
    arena = b["arena"].download(np.uint8, b["arena_bytes"])
    e.tcb_load(tcb, live)
    out = e.alloc(N * 16)
    e.rx_burst_dev(b["arena"].ptr, b["off64"].ptr, b["len"].ptr, N, out.ptr, rxg.REC16)
    e.sync()
    rec = out.download(rxg.REC16_DTYPE, N)
    res[v] = (arena, rec, b["off64"].download(np.uint32, N), b["len"].download(np.uint16, N))
a0, r0, off, lens = res["0"]
a1, r1, _, _ = res["52"]
d = np.nonzero(a0 != a1)[0]
print("arena bytes differ:", len(d), "first", d[:10].tolist())
if len(d):
    fr = np.searchsorted(off.astype(np.int64) * 64, d, side="right") - 1
    u = np.unique(fr)
    print("tx frames differ:", len(u), "slices", np.unique(u // 64)[:20].tolist(), "lanes", np.unique(u % 64)[:64].tolist())
bad = np.nonzero(r0.view(np.uint8).reshape(N, 16).any(axis=1) != 0)[0]
dr = np.nonzero((r0.view(np.uint8).reshape(N, 16) != r1.view(np.uint8).reshape(N, 16)).any(axis=1))[0]
print("rx records differ:", len(dr))
if len(dr):
    print("slices", np.unique(dr // 64)[:30].tolist(), "nslices-range", int(dr.min() // 64), int(dr.max() // 64))
    print("lanes", np.unique(dr % 64).tolist())
    for i in dr[:8]:
        print(int(i), r0[i], r1[i], int(lens[i]))
print("variant-0 verdicts", np.bincount(r0["verdict"], minlength=8).tolist(), "52:", np.bincount(r1["verdict"], minlength=8).tolist())
