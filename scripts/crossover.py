#!/usr/bin/env python3
"""Small-burst crossover: when does routing a burst to rxg beat the
reference's own CPU rx path at its call site (main.c:391-399, MAX_PKT_BURST = 32 at :116)?

rxg side, per burst of n host frames: rxg_rx_burst (views -> pinned staging -> H2D ->
kernel -> D2H records, synchronous) + rxg_rx_replay with empty handlers (the handlers are
the stack's own functions on both sides, so they cancel).  Timed directly at every n.

CPU side: bench.py's CPU-baseline leg (cpu_baseline_per_packet: the oracle's faithful
restatement of the reference path, the only place outside tests/ that runs it) (ARP list walks with
their disabled-logger calls, two-pass linear findtcb with one logger call per scanned TCB,
malloc + memcpy pseudo header and byte-loop checksum), built -O0 (tcp_ip_stack/Makefile:50)
and -O2, in two forms: "shipped" (the reference as it ships: no rx checksum, tcp_in.c:37
if(0)) and "verify" (with the rx checksum rxg computes).  The reference handles one packet
at a time, so its burst time is n x its per-packet time, measured on a bounded sample of the
same frames after one pass has taught its ARP list the sample's sources.

Latency mode (round 3): the same bursts through the persistent server (rxg_server_start;
bursts up to 4 096 frames, 1 and 4 workgroups) are timed beside the launched form.

Prints one JSON line per (frame size, flows) and a summary line with the crossover burst
sizes.  Runs on the GPU box (host cores + one GPU): python scripts/crossover.py [--no-cpu]
"""
import ctypes as C
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dpdk-tcpipstack_amd")]
import torch  # noqa: E402,F401
import bench  # noqa: E402  (its CPU-baseline leg times the reference path)
import rxg  # noqa: E402

BURSTS = [32, 256, 4096, 65536]
# the served bursts, finer around the one-peer crossover (HISTORY.md §6.R3a)
SRV_BURSTS = [32, 64, 96, 128, 160, 192, 256, 4096]
SIZES = [64, 1500]
FLOWS = [1, 1000, 65536]


def rxg_burst_us(eng, lib, views, ptrs, out, n, budget=0.4):
    ops = rxg.HandoffOps()
    # pointers taken once: numpy's .ctypes.data and C.byref cost ~2 us per call in Python,
    # which the stack's own C loop does not pay
    out_p, ops_r = out.ctypes.data, C.byref(ops)
    for _ in range(3):
        lib.rxg_rx_burst(eng.ctx, views, n, rxg.REC8, out_p)
        lib.rxg_rx_replay(eng.ctx, ops_r, ptrs, ptrs, out_p, n, rxg.REC8)
    it, t0 = 0, time.perf_counter()
    while True:
        assert lib.rxg_rx_burst(eng.ctx, views, n, rxg.REC8, out_p) == 0
        assert lib.rxg_rx_replay(eng.ctx, ops_r, ptrs, ptrs, out_p, n, rxg.REC8) == 0
        it += 1
        dt = time.perf_counter() - t0
        if dt > budget and it >= 5:
            return dt / it * 1e6


def main():
    no_cpu = "--no-cpu" in sys.argv
    nmax = max(BURSTS)
    eng = rxg.Engine(0, max_batch=nmax, max_bytes=nmax * 1536)
    lib = rxg.load_library()
    out = np.zeros(nmax, dtype=rxg.REC8_DTYPE)
    rows = []
    for size in SIZES:
        for flows in FLOWS:
            b = eng.synth(n=nmax, nflows=flows, len_a=size, seed=1234 + flows)
            eng.sync()
            off = b["off64"].download(np.uint32, nmax)
            lens = b["len"].download(np.uint16, nmax)
            arena = b["arena"].download(np.uint8, b["arena_bytes"])
            for v in b.values():
                if isinstance(v, rxg.DevArray):
                    v.free()
            tcb, live = rxg.synthetic_tcb_table(flows)
            eng.tcb_load(tcb, live)
            base = arena.ctypes.data
            views = (rxg.PktView * nmax)(*[rxg.PktView(base + int(o) * 64, 0, int(ln), 0) for o, ln in zip(off, lens)])
            ptrs = (C.c_void_p * nmax)(*[base + int(o) * 64 for o in off])
            g = {n: round(rxg_burst_us(eng, lib, views, ptrs, out, n), 1) for n in BURSTS}
            srv = {}
            for blocks in (1, 4):
                eng.server_start(rxg.REC8, blocks=blocks, max_frames=4096)
                srv_dev = eng.server_placement() == rxg.SRV_DEVICE
                srv[blocks] = {n: round(rxg_burst_us(eng, lib, views, ptrs, out, n), 1) for n in SRV_BURSTS}
                eng.server_stop()
            sample = 4096 if flows < 65536 else 1024
            cpu = {}
            for opt in (() if no_cpu else ("O0", "O2")):
                for shipped in (True, False):
                    cpu[f"{opt}_{'shipped' if shipped else 'verify'}"] = round(
                        bench.cpu_baseline_per_packet(arena, off[:sample], lens[:sample], tcb, live, opt, shipped), 4)
            row = {"frame_bytes": size, "flows": flows, "tcbs": flows + 1,
                   "rxg_burst_plus_replay_us": g,
                   "server_burst_plus_replay_us": {f"{b}wg": v for b, v in srv.items()},
                   "rxg_mpps": {n: round(n / g[n], 3) for n in BURSTS},
                   "cpu_us_per_packet": cpu,
                   "cpu_mpps": {k: round(1.0 / v, 4) for k, v in cpu.items()},
                   # smallest measured burst at which rxg's burst time is below the CPU's n x per-packet
                   "crossover_burst": {k: next((n for n in BURSTS if g[n] < n * v), None) for k, v in cpu.items()},
                   "crossover_burst_server": {k: next((n for n in SRV_BURSTS if min(s[n] for s in srv.values()) < n * v), None)
                                              for k, v in cpu.items()},
                   "server_placement": "device staging (large BAR)" if srv_dev else "host staging",
                   "cpu_sample": f"first {sample} frames, ARP list learned from them, 1 core"}
            rows.append(row)
            print(json.dumps(row), flush=True)
    eng.close()
    print(json.dumps({"summary": "crossover burst (rxg burst + replay < reference CPU path), by frame size / flows",
                      "table": {f"{r['frame_bytes']}B_{r['flows']}flows": r["crossover_burst"] for r in rows}}),
          flush=True)


if __name__ == "__main__":
    main()
