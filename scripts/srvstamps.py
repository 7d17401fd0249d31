#!/usr/bin/env python3
"""Where a served burst's device-side microseconds go: the experiment
library's stamping server (RXG_VARIANT 83, rx_server SRVX 8) writes, per request, the
constant-rate wall clock (100 MHz) when workgroup 0 saw the request, after its acquire, after
the rx body, after the record stores landed and after the release, plus the shader clock at
acquire and release (its rate over that span is the clock the body ran at).  Host bursts of
32 x 64 B (rxg_rx_burst, the inline-descriptor form) and device-resident bursts of 32 frames,
each timed on the host too.  Prints one JSON line per case (medians).

  RXG_LIB=dpdk-tcpipstack_amd/rxg/librxg_exp.so RXG_VARIANT=83 python scripts/srvstamps.py"""
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

WALL_MHZ = 100.0  # s_memrealtime


def run(eng, fn, reps=64 * 8):
    """reps calls; the stamps of the last 64 requests and the host's per-call times."""
    for _ in range(64):
        fn()
    host = []
    for _ in range(reps):
        a = time.perf_counter()
        fn()
        host.append(time.perf_counter() - a)
    raw = np.empty(16 + 32 * 8 + 32 * 16, dtype=np.uint64)
    # (a request's stamps reach memory with the next request's release: the last slot may be
    # stale, the medians are over 32)
    eng.d2h(raw.ctypes.data, eng.counters_dev_ptr(), raw.nbytes)
    eng.sync()
    st = raw[16:16 + 256].reshape(32, 8).astype(np.int64)
    bs = raw[16 + 256:].reshape(32, 16).astype(np.int64)  # variant 88: the body's phases
    us = lambda a, b: np.median((st[:, b] - st[:, a]) / WALL_MHZ)  # noqa: E731
    span = (st[:, 4] - st[:, 1]) / WALL_MHZ  # us
    mhz = np.median((st[:, 6] - st[:, 5]) / np.maximum(span, 1e-3))
    extra = {}
    if os.environ["RXG_VARIANT"] == "89":  # the body again right after (code and data cached)
        extra["second_body_us"] = round(float(us(2, 7)), 2)
    if os.environ["RXG_VARIANT"] == "88":
        # body phases from the acquire: frames landed + transposed, fields, probe issued,
        # classified, record put, ring flushed, counters
        names = ["step_entry", "frames_in_lds", "fields", "probe_issued", "classified", "rec_put",
                 "flushed", "counted", "body_entry", "all_small_decided", "frames_issued", "args_built",
                 "class_rounds_done", "class_barrier_passed", "class_classified"]
        for k, nm in enumerate(names):
            extra[nm + "_us"] = round(float(np.median((bs[:, k] - st[:, 1]) / WALL_MHZ)), 2)
        polls = np.maximum(bs[:, 13], 1)
        extra["polls_median"] = int(np.median(bs[:, 13]))
        extra["poll_iteration_us"] = round(float(np.median((st[:, 0] - bs[:, 12]) / WALL_MHZ / polls)), 3)
    return {**extra, "host_us": round(float(np.median(host)) * 1e6, 2),
            "acquire_us": round(float(us(0, 1)), 2), "body_us": round(float(us(1, 2)), 2),
            "stores_landed_us": round(float(us(2, 3)), 2), "release_us": round(float(us(3, 4)), 2),
            "seen_to_released_us": round(float(us(0, 4)), 2), "shader_clock_mhz": round(float(mhz), 0)}


def main():
    if os.environ.get("RXG_VARIANT") not in ("83", "84", "85", "86", "87", "88", "89"):
        sys.exit("srvstamps.py: run with RXG_LIB=<librxg_exp.so> RXG_VARIANT=83 (84: no probe, 85: no stores, "
                 "86: cache-resident buckets, 87: no search, 88: the body's phases, 89: the body twice)")
    n = 256
    eng = rxg.Engine(0, max_batch=n, max_bytes=n * 2048)
    lib = rxg.load_library()
    size = int(os.environ.get("SRVSTAMPS_FRAME", "64"))  # 1500: the class path (the leader and its helpers)
    b = eng.synth(n=n, nflows=1000, len_a=size, seed=5)
    eng.sync()
    off = b["off64"].download(np.uint32, n)
    lens = b["len"].download(np.uint16, n)
    arena = b["arena"].download(np.uint8, b["arena_bytes"])
    tcb, live = rxg.synthetic_tcb_table(1000)
    eng.tcb_load(tcb, live)
    views = (rxg.PktView * n)(*[rxg.PktView(arena.ctypes.data + int(o) * 64, 0, int(ln), 0) for o, ln in zip(off, lens)])
    out = np.zeros(n, dtype=rxg.REC8_DTYPE)
    out_p = out.ctypes.data
    d_out = eng.alloc(n * 8)
    eng.server_start(rxg.REC8, blocks=1, max_frames=n)
    place = {rxg.SRV_DEVICE: "device", rxg.SRV_HOST: "host"}[eng.server_placement()]
    dref = C.byref(rxg.DevBatch(b["arena"].ptr, b["off64"].ptr, b["len"].ptr, 32, rxg.REC8, d_out.ptr))
    for name, fn in ((f"host_32x{size}B_inline", lambda: lib.rxg_rx_burst(eng.ctx, views, 32, rxg.REC8, out_p)),
                     (f"host_33x{size}B", lambda: lib.rxg_rx_burst(eng.ctx, views, 33, rxg.REC8, out_p)),
                     (f"dev_32x{size}B", lambda: lib.rxg_server_burst_dev(eng.ctx, dref))):
        row = {"case": name, "variant": int(os.environ["RXG_VARIANT"]), "placement": place}
        row.update(run(eng, fn))
        print(json.dumps(row), flush=True)
    eng.server_stop()
    d_out.free()
    eng.close()


if __name__ == "__main__":
    main()
