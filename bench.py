#!/usr/bin/env python3
"""bench.py — device-resident rx parse + checksum + classify throughput on MI355X.

Workload (BASELINE.json configs[2], "C3"): 2^20 x 1500 B synthetic Eth/IPv4/TCP frames per
GPU, 1 000 flows + 1 listener, 8-byte records (--rec 16 for the other kind), two rotating
1.5 GiB batches, inputs resident in HBM before timing.  One step = one rxg_rx_burst_dev over the
whole batch.  Legs beside it: C2 64 B frames with a rotating 1 GiB working set
(16 copies of 2^20 frames) so the 256 MiB Infinity Cache cannot hold it, C4 IMIX, the fused
payload hand-off, tx generate, copy-inclusive C3 / C5, burst + replay under churn, small-burst
latency; the CPU baseline at N = 1.

Multi-GPU: one process per GPU (torch.distributed.run), weak scaling, every rank its own
shard (seed + rank) and a replica of the TCB mirror; no data-path collective.  The only
collective is the RCCL all-reduce that merges the per-GPU counters.

Prints ONE JSON line on rank 0 (DESIGN.md §6 for every field).
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
for _p in (ROOT, os.path.join(ROOT, "dpdk-tcpipstack_amd")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import rxg  # noqa: E402  (after torch: one HIP runtime per process)

METRIC = "Mpps + GB/s rx parse+checksum+classify, device-resident, 64B & 1500B frames"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
# Per-launch HBM traffic from the committed rocprofv3 PMC passes of this same command
# (scripts/gpu_prof.sh; scripts/pmc_traffic.py applies the gfx950 FETCH_SIZE x2 fix and stamps
# the src= hash of the build the counted runs loaded: traffic_provenance).  All of round 6's
# tree: REC=8 scripts/gpu_prof.sh ... c3 c2 c2s c4 c2multi c2multis pf3 pr3 tx3 pg3, and
# REC=16 ... c3 c2 c4 c2multi.
TRAFFIC_FILES = {("c3_1500B_1Kflows", 1 << 20, 8): "profiles/r06/c3/traffic.json",
                 ("c2_64B_1flow", 1 << 20, 8): "profiles/r06/c2/traffic.json",
                 ("c4_imix_64Kflows", 1 << 20, 8): "profiles/r06/c4/traffic.json",
                 ("c2_64B_1flow_multiburst", 1 << 20, 8): "profiles/r06/c2multi/traffic.json",
                 ("c2_64B_1flow_strided", 1 << 20, 8): "profiles/r06/c2s/traffic.json",
                 ("c2_64B_1flow_multiburst_strided", 1 << 20, 8): "profiles/r06/c2multis/traffic.json",
                 # the 8(f) kernels over the headline's C3 batch
                 ("tx_generate_dev", 1 << 20, 8): "profiles/r06/tx3/traffic.json",
                 ("payload_gather", 1 << 20, 8): "profiles/r06/pg3/traffic.json",
                 ("c3_rx_payload_fused", 1 << 20, 8): "profiles/r06/pf3/traffic.json",
                 ("c3_rx_payload_by_reference", 1 << 20, 8): "profiles/r06/pr3/traffic.json",
                 # 16-byte records (bench.py --rec 16, and the legs' *_rec16 keys)
                 ("c3_1500B_1Kflows", 1 << 20, 16): "profiles/r06/rec16/c3/traffic.json",
                 ("c2_64B_1flow", 1 << 20, 16): "profiles/r06/rec16/c2/traffic.json",
                 ("c4_imix_64Kflows", 1 << 20, 16): "profiles/r06/rec16/c4/traffic.json",
                 ("c2_64B_1flow_multiburst", 1 << 20, 16): "profiles/r06/rec16/c2multi/traffic.json"}


def traffic_of(name, n, rec):
    """Per-launch HBM bytes of the committed PMC passes of this workload (scripts/gpu_prof.sh),
    or None."""
    tf = TRAFFIC_FILES.get((name, n, rec))
    if tf and os.path.exists(os.path.join(ROOT, tf)):
        with open(os.path.join(ROOT, tf)) as fh:
            return json.load(fh)["hbm_bytes_per_launch"], tf
    return None, None


def traffic_provenance(tf, lib_build: str) -> dict:
    """Whether a traffic file counts the library this process runs: the src= hash its counted
    runs loaded (stamped by scripts/pmc_traffic.py --prov; None for an unstamped file, as every
    file before round 6) against the src= hash of lib_build (rxg_build_info)."""
    stamped = None
    if tf and os.path.exists(os.path.join(ROOT, tf)):
        with open(os.path.join(ROOT, tf)) as fh:
            stamped = json.load(fh).get("source_hash")
    built = next((w[4:] for w in (lib_build or "").split() if w.startswith("src=")), None)
    return {"traffic_src": stamped, "build_src": built,
            "traffic_matches_build": stamped is not None and stamped == built}


WORKLOADS = {
    # name: (frame_len, flows, mix, rotating copies)
    "c3_1500B_1Kflows": (1500, 1000, 0, 2),  # 2 rotating 1.5 GiB batches: no step re-reads the last one's tail from the 256 MB MALL
    "c2_64B_1flow": (64, 1, 0, 16),
    "c4_imix_64Kflows": (0, 65536, 1, 3),
}


# --------------------------------------------------------------- distributed helpers ---
def rank_env():
    return (int(os.environ.get("RANK", 0)), int(os.environ.get("WORLD_SIZE", 1)),
            int(os.environ.get("LOCAL_RANK", 0)))


def shard_seed(base: int, rank: int) -> int:
    """Weak scaling: rank r generates its own independent batch."""
    return (base * 1_000_003 + rank * 7919 + 1) & 0xFFFFFFFFFFFF


def _pg() -> bool:
    """A process group exists: every helper below runs its collective through it, at world
    size 1 too (--pg nccl: the RCCL path exercised on one GPU)."""
    return dist.is_available() and dist.is_initialized()


def merge_counters(counters: np.ndarray, device) -> np.ndarray:
    """Sum the per-GPU counters over ranks (RCCL all-reduce on GPU, gloo on CPU)."""
    if not _pg():
        return counters.copy()
    t = torch.from_numpy(counters.astype(np.int64)).to(device)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return t.cpu().numpy().astype(np.uint64)


def max_over_ranks(x: float, device) -> float:
    if not _pg():
        return x
    t = torch.tensor([x], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def min_over_ranks(x: float, device) -> float:
    if not _pg():
        return x
    t = torch.tensor([x], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MIN)
    return float(t.item())


def sum_over_ranks(x: float, device) -> float:
    if not _pg():
        return x
    t = torch.tensor([float(x)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return float(t.item())


def barrier(device):
    if _pg():
        dist.barrier()
    if torch.cuda.is_available():
        torch.cuda.synchronize()


# ------------------------------------------------------------------------ workload ---
class Workload:
    """`copies` independent synthetic batches of n frames resident in HBM."""

    def __init__(self, eng, name, n, seed, rec=rxg.REC16):
        self.name, self.n, self.rec = name, n, rec
        self.frame_len, self.flows, self.mix, self.copies = WORKLOADS[name]
        self.batches = []
        for c in range(self.copies):
            self.batches.append(eng.synth(n=n, nflows=self.flows, len_a=self.frame_len or 1500,
                                          mix=self.mix, seed=seed + 17 * c))
        eng.sync()
        self.lens = self.batches[0]["len"].download(np.uint16, n)
        self.bytes_per_batch = int(self.lens.astype(np.uint64).sum())
        self.out = eng.alloc(n * rec)

    def launch(self, eng, i, stream=None, strided=False):
        b = self.batches[i % self.copies]
        if strided:  # rxg_rx_bursts_strided_dev: fixed-size frames, frame i at slot i * slots
            eng.rx_bursts_strided_dev(b["arena"].ptr, (self.frame_len + 63) // 64,
                                      [(0, b["len"].ptr, self.n, self.out.ptr)], self.rec, stream)
        else:
            eng.rx_burst_dev(b["arena"].ptr, b["off64"].ptr, b["len"].ptr, self.n, self.out.ptr,
                             self.rec, stream)

    def free(self):
        for b in self.batches:
            for v in b.values():
                if isinstance(v, rxg.DevArray):
                    v.free()
        self.out.free()


def time_workload(eng, wl, steps, warmup, device, stream, strided=False):
    for i in range(warmup):
        wl.launch(eng, i, stream, strided)
    eng.sync()
    eng.counters_reset()
    evs = [(eng.event(), eng.event()) for _ in range(steps)]
    barrier(device)
    t0 = time.perf_counter()
    for i in range(steps):
        eng.record(evs[i][0], stream)
        wl.launch(eng, warmup + i, stream, strided)
        eng.record(evs[i][1], stream)
    eng.sync()
    barrier(device)
    elapsed = time.perf_counter() - t0
    kern_ms = [eng.elapsed_ms(a, b) for a, b in evs]
    for a, b in evs:
        eng.event_destroy(a)
        eng.event_destroy(b)
    return elapsed, kern_ms


def time_region(eng, wl, steps, warmup, device, stream, strided=False):
    """The headline's timed region: `steps` launches back to back on `stream`, one HIP event
    pair around all of them (recorded on that stream), nothing between them.  An event pair
    around every launch adds ~6 us of wall time per launch (scripts/evgap.cpp,
    profiles/r04/evgap/: 250.5 us per C3 launch without events, 256.9 with pairs); the
    per-launch distribution is taken in a separate pass (time_workload).  Returns the host
    wall seconds and the region's event milliseconds."""
    for i in range(warmup):
        wl.launch(eng, i, stream, strided)
    eng.sync()
    eng.counters_reset()
    e0, e1 = eng.event(), eng.event()
    barrier(device)
    t0 = time.perf_counter()
    eng.record(e0, stream)
    for i in range(steps):
        wl.launch(eng, warmup + i, stream, strided)
    eng.record(e1, stream)
    eng.sync()
    barrier(device)
    elapsed = time.perf_counter() - t0
    region_ms = eng.elapsed_ms(e0, e1)
    eng.event_destroy(e0)
    eng.event_destroy(e1)
    return elapsed, region_ms


def multiburst_leg(eng, steps, warmup, device, seed, nbursts=16, n=1 << 20, rec=rxg.REC16, strided=False):
    """C2 (configs[1]: 2^20 x 64 B, 1 flow) as a ring of `nbursts` distinct 2^20-frame bursts
    in one 1 GiB frame pool (the same working set as the rotating C2 leg, beyond the 256 MB
    Infinity Cache), classified by ONE launch (rxg_rx_bursts_dev) instead of one launch per
    burst: the launch ramp and drain are paid once per ring.  Roofline per launch =
    nbursts x 64 MiB of frame bytes / (the launches' event time / launches)."""
    pool = eng.synth(n=n * nbursts, nflows=1, len_a=64, mix=0, seed=seed + 123)
    tcb, live = rxg.synthetic_tcb_table(1)
    eng.tcb_load(tcb, live)
    out = eng.alloc(n * nbursts * rec)
    bursts = [(pool["off64"].ptr + j * n * 4, pool["len"].ptr + j * n * 2, n, out.ptr + j * n * rec)
              for j in range(nbursts)]
    # strided: the same frames through rxg_rx_bursts_strided_dev (burst j's frame i at slot j n + i)
    sbursts = [(j * n, pool["len"].ptr + j * n * 2, n, out.ptr + j * n * rec) for j in range(nbursts)]

    def launch():
        if strided:
            eng.rx_bursts_strided_dev(pool["arena"].ptr, 1, sbursts, rec)
        else:
            eng.rx_bursts_dev(pool["arena"].ptr, bursts, rec)
    try:
        for _ in range(warmup):
            launch()
        eng.sync()
        eng.counters_reset()
        e0, e1 = eng.event(), eng.event()
        barrier(device)
        t0 = time.perf_counter()
        eng.record(e0)  # one event pair around the launches (time_region)
        for _ in range(steps):
            launch()
        eng.record(e1)
        eng.sync()
        barrier(device)
        dt = max_over_ranks(time.perf_counter() - t0, device)
        k = max_over_ranks(eng.elapsed_ms(e0, e1) / steps / 1e3, device)
        eng.event_destroy(e0)
        eng.event_destroy(e1)
        c = merge_counters(eng.counters(), device)
        frames_all = int(sum_over_ranks(n * nbursts, device)) * steps
        alg = n * nbursts * 64
        last = out.download(rxg.rec_dtype(rec), 4096, offset_bytes=(n * nbursts - 4096) * rec)
        if rec == rxg.REC8:
            last = rxg.rec8_expand(last)
        return {"bursts_per_launch": nbursts, "frames_per_burst": n, "rec_kind": rec,
                "descriptors": "fixed stride (no off64[])" if strided else "off64[] + len[]",
                "traffic_bytes_per_launch": traffic_of("c2_64B_1flow_multiburst" + ("_strided" if strided else ""),
                                                       n, rec)[0],
                "algorithmic_bytes_per_launch": alg,
                "kernel_us_per_launch": round(k * 1e6, 2), "kernel_us_per_burst": round(k * 1e6 / nbursts, 2),
                "mpps": round(frames_all / dt / 1e6, 2), "gbs": round(frames_all * 64 / dt / 1e9, 2),
                "roofline_frac": round(alg / k / 1e9 / HBM_PEAK_GBS, 4), "working_set_GiB": round(alg / 2**30, 3),
                "counters_ok": bool(int(c[0]) == frames_all and int(c[7]) == 0 and int(c[8]) == 0
                                    and int(c[13]) == frames_all
                                    and (last["verdict"] == rxg.V_DISPATCH).all() and (last["tcb_idx"] == 1).all())}
    finally:
        out.free()
        for v in pool.values():
            if isinstance(v, rxg.DevArray):
                v.free()


def copy_inclusive_leg(eng, wl, steps, warmup, device):
    """The path as it runs from host mbufs: pinned H2D of the packed batch (arena +
    descriptors), the rx kernel, D2H of the records; one stream, back to back.  PCIe-bound;
    reported beside `value`, never as it."""
    b = wl.batches[0]
    nb = b["arena_bytes"]
    h_arena, h_off, h_len = eng.pinned(nb), eng.pinned(wl.n * 4), eng.pinned(wl.n * 2)
    h_out = eng.pinned(wl.n * wl.rec)
    eng.d2h(h_arena.ptr, b["arena"].ptr, nb)
    eng.d2h(h_off.ptr, b["off64"].ptr, wl.n * 4)
    eng.d2h(h_len.ptr, b["len"].ptr, wl.n * 2)
    eng.sync()
    d_arena, d_off, d_len = eng.alloc(nb), eng.alloc(wl.n * 4), eng.alloc(wl.n * 2)

    def step():
        eng.h2d(d_arena.ptr, h_arena.ptr, nb)
        eng.h2d(d_off.ptr, h_off.ptr, wl.n * 4)
        eng.h2d(d_len.ptr, h_len.ptr, wl.n * 2)
        eng.rx_burst_dev(d_arena.ptr, d_off.ptr, d_len.ptr, wl.n, wl.out.ptr, wl.rec)
        eng.d2h(h_out.ptr, wl.out.ptr, wl.n * wl.rec)

    for _ in range(warmup):
        step()
    eng.sync()
    barrier(device)
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    eng.sync()
    barrier(device)
    dt = max_over_ranks(time.perf_counter() - t0, device)
    res = {"mpps": round(sum_over_ranks(wl.n, device) * steps / dt / 1e6, 2),
           "gbs": round(sum_over_ranks(wl.bytes_per_batch, device) * steps / dt / 1e9, 2),
           "h2d_bytes_per_step": nb + wl.n * 6, "d2h_bytes_per_step": wl.n * wl.rec,
           "ms_per_step": round(dt / steps * 1e3, 3)}
    for a in (h_arena, h_off, h_len, h_out):
        a.free()
    for a in (d_arena, d_off, d_len):
        a.free()
    return res


def c5_leg(eng, n, steps, warmup, device, seed):
    """Config 5: bidirectional, copy-inclusive, 2^20 flows, one GPU's share (weak scaling).
    tx: host-built IMIX frames in pinned host memory; the checksum-generate kernel (ip_out,
    ip.c:97-118) reads them over PCIe and writes each frame's patched first line back in
    place (zero-copy: no staging copy, and 64 B instead of the whole frame come back).
    rx: host frames -> H2D -> parse+verify+classify -> D2H of the records.  tx and rx run
    on two HIP streams.  scripts/zcbench.py c5 compares the variants (copies both ways on
    one or two streams, zero-copy both)."""
    flows = 1 << 20
    tx = eng.synth(n=n, nflows=flows, mix=1, seed=seed + 5)
    rx = eng.synth(n=n, nflows=flows, mix=1, seed=seed + 6)
    eng.sync()
    tcb, live = rxg.synthetic_tcb_table(flows)
    eng.tcb_load(tcb, live)
    eng.tcb_sync()
    nb = tx["arena_bytes"]
    lens = rx["len"].download(np.uint16, n)
    tx_lens = tx["len"].download(np.uint16, n)
    host = {k: eng.pinned(v) for k, v in (("tx", nb), ("rx", rx["arena_bytes"]), ("txo", n * 4),
                                           ("txl", n * 2), ("rxo", n * 4), ("rxl", n * 2),
                                           ("rec", n * 16))}
    eng.d2h(host["tx"].ptr, tx["arena"].ptr, nb)
    eng.d2h(host["rx"].ptr, rx["arena"].ptr, rx["arena_bytes"])
    for k, d, sz in (("txo", tx["off64"], n * 4), ("txl", tx["len"], n * 2),
                     ("rxo", rx["off64"], n * 4), ("rxl", rx["len"], n * 2)):
        eng.d2h(host[k].ptr, d.ptr, sz)
    eng.sync()
    out = eng.alloc(n * 16)
    # the host frames start without checksums (ip_out sums the fields as zero)
    t_off = host["txo"].np[: n * 4].view(np.uint32).astype(np.int64) * 64
    for bpos in (24, 25, 50, 51):
        host["tx"].np[t_off + bpos] = 0
    s_tx = torch.cuda.Stream(device=eng.device)
    st = s_tx.cuda_stream  # tx direction; rx on the engine's own stream

    def step():
        eng.tx_cksum_dev(host["tx"].ptr, host["txo"].ptr, host["txl"].ptr, n, st)
        eng.h2d(rx["arena"].ptr, host["rx"].ptr, rx["arena_bytes"])
        eng.h2d(rx["off64"].ptr, host["rxo"].ptr, n * 4)
        eng.h2d(rx["len"].ptr, host["rxl"].ptr, n * 2)
        eng.rx_burst_dev(rx["arena"].ptr, rx["off64"].ptr, rx["len"].ptr, n, out.ptr, 16)
        eng.d2h(host["rec"].ptr, out.ptr, n * 16)

    def sync_both():
        eng.sync()
        eng.stream_sync(st)

    for _ in range(warmup):
        step()
    sync_both()
    eng.counters_reset()
    barrier(device)
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    sync_both()
    barrier(device)
    dt = max_over_ranks(time.perf_counter() - t0, device)
    c = merge_counters(eng.counters(), device)
    # the host tx frames now carry exactly the checksums the synthetic generator computed
    ref = tx["arena"].download(np.uint8, nb)
    tx_ok = bool(np.array_equal(host["tx"].np[:nb], ref))
    rec = host["rec"].np[: n * 16].view(rxg.REC16_DTYPE)
    n_all = int(sum_over_ranks(n, device))
    b_all = sum_over_ranks(int(lens.astype(np.uint64).sum()) + int(tx_lens.astype(np.uint64).sum()), device)
    ok = bool((rec["verdict"] == rxg.V_DISPATCH).all() and (rec["tcp_cksum"] == 0).all()
              and int(c[0]) == n_all * steps and int(c[8]) == 0 and tx_ok)
    res = {"frames_per_dir_per_gpu": n, "flows": flows, "frame_mix": "imix 64/576/1500 7:4:1",
           "mpps_per_direction": round(n_all * steps / dt / 1e6, 2),
           "gbs_both_directions": round(b_all * steps / dt / 1e9, 2),
           "ms_per_step": round(dt / steps * 1e3, 3), "counters_ok": ok}
    for a in host.values():
        a.free()
    for d in list(tx.values()) + list(rx.values()) + [out]:
        if isinstance(d, rxg.DevArray):
            d.free()
    return res


def payload_leg(eng, wl, steps, warmup):
    """the device payload gather (rxg_payload_gather_dev) after a burst
    of the workload.  Algorithmic bytes per launch = 2 x payload bytes (read + write) + the
    record read (wl.rec bytes) + 16 B descriptor write per frame; HIP events around the three
    launches."""
    wl.launch(eng, 0)
    pl = (wl.lens.astype(np.int64) - 54).clip(min=0)  # synthetic frames: IHL 5, data_off 5
    dl = int(pl.sum())
    cap = int(((pl + 15) // 16 * 16).sum())
    arena, msgs, used = eng.alloc(cap), eng.alloc(wl.n * 16), eng.alloc(8)
    try:
        for _ in range(warmup):
            eng.payload_gather_dev(arena.ptr, cap, msgs.ptr, used.ptr)
        evs = [(eng.event(), eng.event()) for _ in range(steps)]
        for a, b in evs:
            eng.record(a)
            eng.payload_gather_dev(arena.ptr, cap, msgs.ptr, used.ptr)
            eng.record(b)
        eng.sync()
        ms = [eng.elapsed_ms(a, b) for a, b in evs]
        k = float(np.mean(ms)) / 1e3
        alg = 2 * dl + (wl.rec + 16) * wl.n
        assert int(used.download(np.uint64, 1)[0]) == cap
        tb = traffic_of("payload_gather", wl.n, wl.rec)[0] if wl.name == "c3_1500B_1Kflows" else None
        return {"payload_bytes": dl, "arena_bytes": cap, "record_bytes": wl.rec,
                "traffic_bytes_per_launch": tb,
                "kernels_us": round(k * 1e6, 2), "achieved_GBps": round(alg / k / 1e9, 1),
                "roofline_frac": round(alg / k / 1e9 / HBM_PEAK_GBS, 4),
                "algorithmic_bytes_per_launch": alg}
    finally:
        for d in (arena, msgs, used):
            d.free()


def fused_leg(eng, wl, steps, warmup, by_reference=False):
    """The burst and its payload hand-off in ONE pass (rxg_rx_burst_payload_dev, DESIGN.md
    §5.F) over the workload's rotating batches, against the two-pass form (rxg_rx_burst_dev,
    then rxg_payload_gather_dev reading every payload byte again).  One event pair around the
    launches.  Algorithmic bytes per launch = the frame bytes read + the payload bytes handed
    off + a 16-byte message and a record per frame (the two-pass form moves the same plus
    the payload read a second time)."""
    # by_reference: no arena -- each message names its payload in the pool itself (nothing
    # copied; rxg.h rxg_rx_burst_payload_dev), the algorithmic bytes without the payload write
    arenas = [None if by_reference else eng.alloc(b["arena_bytes"]) for b in wl.batches]
    msgs = eng.alloc(wl.n * 16)
    pl = (wl.lens.astype(np.int64) - 54).clip(min=0)  # synthetic frames: IHL 5, data_off 5
    dl = int(pl.sum())
    try:
        def launch(i):
            b = wl.batches[i % wl.copies]
            ar = arenas[i % wl.copies]
            eng.rx_burst_payload_dev(b["arena"].ptr, b["off64"].ptr, b["len"].ptr, wl.n, wl.out.ptr,
                                     ar.ptr if ar else None, msgs.ptr, wl.rec)
        for i in range(warmup):
            launch(i)
        eng.sync()
        eng.counters_reset()
        e0, e1 = eng.event(), eng.event()
        eng.record(e0)
        for i in range(steps):
            launch(warmup + i)
        eng.record(e1)
        eng.sync()
        k = eng.elapsed_ms(e0, e1) / steps / 1e3
        eng.event_destroy(e0)
        eng.event_destroy(e1)
        c = eng.counters()
        m = msgs.download(rxg.PAYLOAD_MSG_DTYPE, wl.n)
        alg = wl.bytes_per_batch + (0 if by_reference else dl) + (16 + wl.rec) * wl.n
        tb = (traffic_of("c3_rx_payload_by_reference" if by_reference else "c3_rx_payload_fused", wl.n, wl.rec)[0]
              if wl.name == "c3_1500B_1Kflows" else None)
        return {"kernel_us": round(k * 1e6, 2), "mpps": round(wl.n / k / 1e6, 1),
                "payload_bytes": dl, "algorithmic_bytes_per_launch": alg,
                "traffic_bytes_per_launch": tb,
                "achieved_GBps": round(alg / k / 1e9, 1), "roofline_frac": round(alg / k / 1e9 / HBM_PEAK_GBS, 4),
                "ok": bool(int(c[0]) == wl.n * steps and int(c[13]) == wl.n * steps and int(c[8]) == 0
                           and (m["len"] == pl).all())}
    finally:
        for d in arenas + [msgs]:
            if d is not None:
                d.free()


def tx_leg(eng, wl, steps, warmup):
    """tx checksum generate (rxg_tx_cksum_dev, what ip_out computes,
    ip.c:97-118) over the device-resident batch of the workload, in place.  The frames'
    checksums are already the generated values, so the batch stays valid.  Algorithmic
    bytes per launch = the frame bytes read (the 4 checksum bytes written per frame are
    included in the traffic, not in the unit)."""
    b = wl.batches[0]
    for _ in range(warmup):
        eng.tx_cksum_dev(b["arena"].ptr, b["off64"].ptr, b["len"].ptr, wl.n)
    evs = [(eng.event(), eng.event()) for _ in range(steps)]
    for a, e in evs:
        eng.record(a)
        eng.tx_cksum_dev(b["arena"].ptr, b["off64"].ptr, b["len"].ptr, wl.n)
        eng.record(e)
    eng.sync()
    k = float(np.mean([eng.elapsed_ms(a, e) for a, e in evs])) / 1e3
    tb = traffic_of("tx_generate_dev", wl.n, wl.rec)[0] if wl.name == "c3_1500B_1Kflows" else None
    return {"kernel_us": round(k * 1e6, 2), "mpps": round(wl.n / k / 1e6, 1),
            "algorithmic_bytes_per_launch": wl.bytes_per_batch, "traffic_bytes_per_launch": tb,
            "achieved_GBps": round(wl.bytes_per_batch / k / 1e9, 1),
            "roofline_frac": round(wl.bytes_per_batch / k / 1e9 / HBM_PEAK_GBS, 4)}


# Rank 0 runs the replay_churn and small_burst legs alone while the other ranks wait at the
# next barrier: together they may take at most this long (subprocess time limits), far below
# --pg-timeout, so no waiting rank's collective can time out on them.
SOLO_BUDGET_S = 180.0


def replay_churn_leg(deadline=None):
    """SURVEY.md 8(f) row 2 under load: burst + in-order replay (rxg_rx_replay) with C
    handlers shaped like tcp_states.c's, 1 % of the frames starting a connection event (a new
    client's SYN + ACK: tcp_listen appends a child, tcp_syn_rcv establishes it; or an
    established flow's FIN + next segment: CLOSED, then remove_tcb), at the C4 and C5 table
    sizes, 4 096-frame bursts of 64 B frames, beside the same run without churn.  Runs
    dpdk-tcpipstack_amd/build/churn_bench (a child process on the same GPU)."""
    import subprocess
    exe = os.path.join(ROOT, "dpdk-tcpipstack_amd", "build", "churn_bench")
    if not os.path.exists(exe):
        return None
    out = {}
    deadline = deadline or time.perf_counter() + SOLO_BUDGET_S
    for nflows in (65536, 1 << 20):
        for permille in (0, 10):
            left = deadline - time.perf_counter()
            if left < 5:
                return dict(out, error="solo-leg budget spent")
            try:
                r = subprocess.run([exe, str(nflows), "4096", "40", str(permille)], capture_output=True,
                                   text=True, timeout=left)
            except subprocess.TimeoutExpired:
                return dict(out, error=f"churn_bench exceeded the solo-leg budget ({SOLO_BUDGET_S:g} s)")
            if r.returncode != 0:
                return {"error": r.stderr.strip()[-300:]}
            d = json.loads(r.stdout)
            out[f"tcbs_{nflows + 1}_churn_{permille / 10:g}pct"] = {
                k: d[k] for k in ("burst_us", "d2h_us", "replay_us", "mpps_with_replay", "stale_per_burst",
                                  "host_fixups_per_burst", "device_launches_per_burst", "ntcb_end")}
    return out


def small_burst_leg(gpu, n=32, seconds=0.3):
    """SURVEY.md 8(a) A1 at the reference's own burst size (MAX_PKT_BURST = 32, main.c:116):
    host frames through rxg_rx_burst + rxg_rx_replay (empty handlers), median microseconds per
    burst, launched and through the latency-mode server (rxg_server_start),
    64 B and 1 500 B frames, 1 000 flows, 8-byte records."""
    import ctypes as C
    e = rxg.Engine(device=gpu, max_batch=4096, max_bytes=4096 * 1536)
    lib = rxg.load_library()
    out = np.zeros(n, dtype=rxg.REC8_DTYPE)
    ops = rxg.HandoffOps()
    res = {}
    try:
        for size in (64, 1500):
            b = e.synth(n=n, nflows=1000, len_a=size, seed=4242)
            e.sync()
            off = b["off64"].download(np.uint32, n)
            lens = b["len"].download(np.uint16, n)
            arena = b["arena"].download(np.uint8, b["arena_bytes"])
            for v in b.values():
                if isinstance(v, rxg.DevArray):
                    v.free()
            tcb, live = rxg.synthetic_tcb_table(1000)
            e.tcb_load(tcb, live)
            base = arena.ctypes.data
            views = (rxg.PktView * n)(*[rxg.PktView(base + int(o) * 64, 0, int(ln), 0) for o, ln in zip(off, lens)])
            ptrs = (C.c_void_p * n)(*[base + int(o) * 64 for o in off])

            # pointers taken once: numpy's .ctypes.data and C.byref cost ~2 us per call in
            # Python, which the stack's own C loop does not pay
            out_p, ops_r = out.ctypes.data, C.byref(ops)

            def one():
                t = time.perf_counter()
                assert lib.rxg_rx_burst(e.ctx, views, n, rxg.REC8, out_p) == 0
                assert lib.rxg_rx_replay(e.ctx, ops_r, ptrs, ptrs, out_p, n, rxg.REC8) == 0
                return time.perf_counter() - t

            def median_us():
                for _ in range(5):
                    one()
                lat, t0 = [], time.perf_counter()
                while time.perf_counter() - t0 < seconds or len(lat) < 20:
                    lat.append(one())
                return round(float(np.median(lat)) * 1e6, 2)
            launched = median_us()
            e.server_start(rxg.REC8, blocks=4, max_frames=4096)
            served = median_us()
            e.server_stop()
            res[f"{size}B_x{n}"] = {"launched_us": launched, "served_us": served,
                                    "served_mpps": round(n / served, 3)}
    finally:
        e.close()
    return res


def host_cpus() -> dict:
    """The host the CPU baseline runs on: the CPU model, nproc, this
    process's affinity, and the cgroup CPU quota (cpu.max) when one is set -- on the GPU box
    nproc and the affinity show the whole machine while the job's share is smaller.  `usable`
    = the affinity, capped by that share: the replica leg's core count."""
    model = None
    try:
        with open("/proc/cpuinfo") as fh:
            model = next((ln.split(":", 1)[1].strip() for ln in fh if ln.startswith("model name")), None)
    except OSError:
        pass
    aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as fh:
            q, per = fh.read().split()[:2]
        if q != "max":
            quota = int(q) / int(per)
    except (OSError, ValueError):
        pass
    # the job's CPU share: the cgroup quota, else the thread budget the job was given
    # (OMP_NUM_THREADS: 16 per GPU on the GPU box, whose affinity spans the whole machine)
    omp = os.environ.get("OMP_NUM_THREADS", "")
    if quota is not None:
        usable, why = max(1, min(aff, int(quota))), "cgroup cpu.max quota"
    elif omp.isdigit() and int(omp) > 0:
        usable, why = min(aff, int(omp)), "OMP_NUM_THREADS (the job's thread budget)"
    else:
        usable, why = aff, "affinity"
    return {"model": model, "nproc": os.cpu_count(), "affinity": aff,
            "cgroup_quota_cpus": round(quota, 2) if quota is not None else None,
            "omp_num_threads": int(omp) if omp.isdigit() else None, "usable": usable, "usable_from": why}


def cpu_baseline(eng, wl, seconds=10.0, sample_n=20000, cores=1):
    """The oracle's faithful restatement of the reference rx path (port), on one host
    core, over a bounded sample of the same workload (first sample_n frames)."""
    import oracle
    b = wl.batches[0]
    n = min(sample_n, wl.n)
    off = b["off64"].download(np.uint32, n)
    lens = b["len"].download(np.uint16, n)
    end = int(off[-1]) * 64 + int(lens[-1])
    arena = b["arena"].download(np.uint8, (end + 63) // 64 * 64)
    tcb, live = rxg.synthetic_tcb_table(wl.flows)
    res = {}
    for opt, budget in (("O0", seconds * 0.5), ("O2", seconds * 0.5)):
        oracle.arp_reset()
        oracle.rx_batch(arena, off, lens, tcb, live, faithful=True, opt=opt)  # learn ARP
        pk = by = 0
        t0 = time.perf_counter()
        chunk = max(64, min(n, 2000))
        s = 0
        while time.perf_counter() - t0 < budget:
            e = min(s + chunk, n)
            oracle.rx_batch(arena, off[s:e], lens[s:e], tcb, live, faithful=True, opt=opt)
            pk += e - s
            by += int(lens[s:e].astype(np.uint64).sum())
            s = 0 if e >= n else e
        dt = time.perf_counter() - t0
        res[opt] = (pk / dt / 1e6, by / dt / 1e9, pk, dt)
        arp_entries = oracle.arp_count(opt)  # the list each packet's get_mac walks (ip.c:26-32)
    oracle.arp_reset()
    mpps0, gbs0, pk0, dt0 = res["O0"]
    mpps2, gbs2, pk2, dt2 = res["O2"]
    multi = cpu_replicas(arena, off, lens, tcb, live, cores, seconds * 0.5) if cores > 1 else None
    if multi:
        multi["per_core_over_1core_O0"] = round(multi["mpps"] / multi["cores"] / mpps0, 3)
    # SURVEY.md §6 timed the reference's own hot-path files on this shape (1 500 B, 1 000 flows /
    # 1 000 source IPs, +verify) in the survey's container: 0.0121 Mpps at -O0, 0.0185 at -O2.
    # The port, timed on the same shape in the same container class (scripts/cpu_calib.py,
    # profiles/r05/cpu_calib/container.json), runs 1.37x (-O0) / 1.5x (-O2) slower; no slower
    # construct was found in its code (HISTORY.md §6.R5), and the reference cannot be built here
    # (no DPDK headers) to time it on this host.  So the factor is stated, with the reference-
    # equivalent rate it implies: a GPU-over-CPU ratio against `value` is inflated by it.
    calib = None
    cf = os.path.join(ROOT, "profiles", "r05", "cpu_calib", "container.json")
    if wl.name == "c3_1500B_1Kflows" and os.path.exists(cf):
        with open(cf) as fh:
            cc = json.load(fh)
        f0, f2 = cc["reference_over_port_O0"], cc["reference_over_port_O2"]
        calib = {"source": "profiles/r05/cpu_calib/container.json (scripts/cpu_calib.py)",
                 "shape": cc["shape"], "reference_over_port": {"O0": f0, "O2": f2},
                 "reference_equivalent": {"O0_mpps": round(mpps0 * f0, 6), "O0_gbs": round(gbs0 * f0, 6),
                                          "O2_mpps": round(mpps2 * f2, 6), "O2_gbs": round(gbs2 * f2, 6)}}
    return {"value": round(gbs0, 6), "unit": "GB/s", "mpps": round(mpps0, 6), "cores": 1,
            "kind": "port", "host": host_cpus(), "arp_entries": arp_entries,
            "sample": (f"faithful oracle (reference algorithms: byte-loop checksum, malloc+memcpy "
                       f"pseudo header, two-pass linear findtcb over {wl.flows + 1} TCBs, ARP list "
                       f"walks, disabled-logger calls) built -O0 like tcp_ip_stack/Makefile:50, "
                       f"{pk0} frames of this workload in {dt0:.1f} s on 1 core; "
                       f"-O2 build: {mpps2:.4f} Mpps / {gbs2:.4f} GB/s"
                       + (f"; the reference's own files ran {calib['reference_over_port']['O0']}x (-O0) / "
                          f"{calib['reference_over_port']['O2']}x (-O2) this port's rate on this shape in the "
                          f"survey's container (calibration.reference_equivalent)" if calib else "")),
            "o2": {"mpps": round(mpps2, 6), "gbs": round(gbs2, 6)},
            "calibration": calib,
            "replicas": multi}


def cpu_baseline_per_packet(arena, off, lens, tcb, live, opt, shipped, budget=1.0):
    """The CPU baseline per packet at the reference's call site (scripts/crossover.py, DESIGN.md
    §6.R3a): the faithful oracle (-O0 / -O2; shipped = the reference's rx checksum compiled
    out, tcp_in.c:37) over the given frames in bursts of 64, after one pass has taught its ARP
    list their sources; microseconds per packet on one host core."""
    import oracle
    oracle.arp_reset()
    oracle.rx_batch(arena, off, lens, tcb, live, faithful=True, opt=opt, shipped=shipped)  # learn ARP
    n, pk, s, t0 = len(lens), 0, 0, time.perf_counter()
    while time.perf_counter() - t0 < budget or pk == 0:
        e = min(s + 64, n)
        oracle.rx_batch(arena, off[s:e], lens[s:e], tcb, live, faithful=True, opt=opt, shipped=shipped)
        pk += e - s
        s = 0 if e >= n else e
    dt = time.perf_counter() - t0
    oracle.arp_reset()
    return dt / pk * 1e6


def cpu_replicas(arena, off, lens, tcb, live, cores, seconds):
    """one independent replica of the faithful oracle (-O0) per host
    core, each its own process with private tables, on disjoint ranges of the sample.
    Child processes only: nothing here touches the GPU."""
    import subprocess
    import tempfile
    n = len(lens)
    cores = max(1, min(cores, n))
    with tempfile.TemporaryDirectory() as td:
        path = os.path.join(td, "sample.npz")
        np.savez(path, arena=arena, off=off, lens=lens, tcb=tcb, live=live)
        cuts = [n * k // cores for k in range(cores + 1)]
        procs = [subprocess.Popen([sys.executable, os.path.join(ROOT, "oracle", "replica.py"), path,
                                   str(cuts[k]), str(cuts[k + 1]), str(seconds), "O0"],
                                  stdout=subprocess.PIPE, text=True) for k in range(cores)]
        try:
            outs = [json.loads(p.communicate(timeout=seconds + 120)[0]) for p in procs]
        except (ValueError, subprocess.TimeoutExpired):  # a replica died: report no figure
            for p in procs:
                p.kill()
            return None
    if any(p.returncode for p in procs):
        return None
    mpps = sum(o["frames"] / o["seconds"] for o in outs) / 1e6
    gbs = sum(o["bytes"] / o["seconds"] for o in outs) / 1e9
    arp = sorted({o["arp_entries"] for o in outs})
    return {"cores": cores, "mpps": round(mpps, 6), "gbs": round(gbs, 6), "opt": "O0",
            "arp_entries": arp[0] if len(arp) == 1 else arp,
            "sample": f"{cores} processes (one per usable core: host.usable), frames split "
                      f"{cuts[1] - cuts[0]}-ish each, each after an untimed pass over the whole sample "
                      f"(its ARP list = the 1-core leg's), {seconds:.1f} s"}


def _free_port() -> int:
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(ngpus: int) -> int:
    """`python bench.py --gpus N` (N > 1) with no launcher around it: start N fresh rank
    processes through torch.distributed.run (one per GPU, rendezvous on 127.0.0.1) as a
    CHILD process and return its exit code.  Nothing here touches the GPU (device_count does
    not initialise it on this image), and the parent never execs.  The ranks are this same
    script with the same arguments; they see WORLD_SIZE and run main's rank path."""
    import subprocess
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={ngpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("OMP_NUM_THREADS", "1")  # torch.distributed.run's own default, without its warning
    return subprocess.run(cmd, env=env).returncode


def pg_backend(pg: str, world: int, rehearse: bool):
    """The process group's backend, or None for no process group (--pg auto at world 1)."""
    if pg == "auto":
        return None if world == 1 else ("gloo" if rehearse else "nccl")
    return pg


def init_pg(backend: str, rank: int, world: int, timeout_s: float) -> None:
    """init_process_group with an explicit timeout: no collective (and no rank waiting at a
    barrier for rank 0's solo legs) waits longer than timeout_s.  At world 1 without a
    launcher the rendezvous is this process alone, on 127.0.0.1."""
    import datetime
    if "MASTER_ADDR" not in os.environ:
        os.environ["MASTER_ADDR"] = "127.0.0.1"
    if "MASTER_PORT" not in os.environ:
        os.environ["MASTER_PORT"] = str(_free_port())
    os.environ.setdefault("RANK", str(rank))
    os.environ.setdefault("WORLD_SIZE", str(world))
    dist.init_process_group(backend, init_method="env://", rank=rank, world_size=world,
                            timeout=datetime.timedelta(seconds=timeout_s))


def rank_devices(gpu: int, have_gpu: bool, device) -> list:
    """Every rank's device as the rank itself sees it (gathered to all ranks): what the line's
    n_gpus / ranks were measured on."""
    me = {"rank": int(os.environ.get("RANK", 0)), "device": f"cuda:{gpu}" if have_gpu else "cpu"}
    if have_gpu:
        p = torch.cuda.get_device_properties(gpu)
        me["name"] = p.name
        uuid = getattr(p, "uuid", None)
        if uuid is not None:
            me["uuid"] = str(uuid)
    if not _pg():
        return [me]
    out = [None] * dist.get_world_size()
    dist.all_gather_object(out, me)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--workload", default="c3_1500B_1Kflows", choices=sorted(WORKLOADS))
    ap.add_argument("--frames", type=int, default=1 << 20, help="frames per GPU per step")
    # record kind: 8 = rxg_rec8, everything rxg_rx_replay and the payload gather read
    # (checksums as ok bits); 16 / 48 carry the checksum values / every header field
    ap.add_argument("--rec", type=int, default=8, choices=[8, 16, 48])
    ap.add_argument("--no-legs", action="store_true", help="skip the 64 B / IMIX legs")
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline leg")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--cpu-cores", type=int, default=0,
                    help="replicas for the multi-core CPU leg (0: this process's CPU share, at most 16)")
    ap.add_argument("--scaling", default="weak", choices=["weak", "strong"],
                    help="weak: --frames per GPU; strong: --total-frames split over the GPUs")
    ap.add_argument("--total-frames", type=int, default=1 << 23)
    # auto: a process group only when WORLD_SIZE > 1 (nccl = RCCL; gloo when rehearsing).
    # nccl / gloo: that backend at every world size, 1 included, so the RCCL init,
    # all_reduce, all_gather_object, barrier and destroy run on one GPU before any N > 1 run.
    ap.add_argument("--pg", default=os.environ.get("RXG_BENCH_PG", "auto"), choices=["auto", "nccl", "gloo"])
    ap.add_argument("--pg-timeout", type=float, default=900.0,
                    help="seconds any collective may wait (init_process_group timeout)")
    args = ap.parse_args()
    if args.gpus < 1:
        sys.exit(f"bench.py: --gpus {args.gpus}: need at least 1")

    # RXG_BENCH_REHEARSE=1: rehearse N ranks on fewer GPUs (device = local_rank mod #GPUs,
    # gloo backend for the collectives) -- a correctness rehearsal, never a measurement.
    rehearse = os.environ.get("RXG_BENCH_REHEARSE") == "1"
    if "WORLD_SIZE" not in os.environ:
        if args.gpus > 1:
            ndev = torch.cuda.device_count()
            if not rehearse and ndev < args.gpus:
                sys.exit(f"bench.py: --gpus {args.gpus} but {ndev} GPU(s) visible "
                         "(RXG_BENCH_REHEARSE=1 rehearses more ranks than GPUs)")
            sys.exit(spawn_ranks(args.gpus))
    elif int(os.environ["WORLD_SIZE"]) != args.gpus:
        sys.exit(f"bench.py: launched with WORLD_SIZE={os.environ['WORLD_SIZE']} but --gpus {args.gpus}")

    rank, world, local = rank_env()
    have_gpu = torch.cuda.device_count() > 0
    gpu = local % max(1, torch.cuda.device_count()) if rehearse else local
    backend = pg_backend(args.pg, world, rehearse)
    if backend:
        if have_gpu:
            torch.cuda.set_device(gpu)
        init_pg(backend, rank, world, args.pg_timeout)
    # the collectives' tensors live where the backend reduces them (RCCL: the GPU)
    device = torch.device("cuda", gpu) if backend == "nccl" or (have_gpu and not backend) else torch.device("cpu")
    ranks = dist.get_world_size() if dist.is_initialized() else 1
    devices = rank_devices(gpu, have_gpu, device)
    if not have_gpu:
        if not rehearse:
            sys.exit("bench.py: no GPU visible")
        # rehearsal on a host without a GPU: the launcher, the rendezvous and the collectives
        # only; nothing is measured, so the line carries no value
        t = max_over_ranks(float(rank + 1), device)
        if rank == 0:
            print(json.dumps({"metric": METRIC, "value": None, "unit": "GB/s", "n_gpus": world, "ranks": ranks,
                              "devices": devices, "rehearsal": "no GPU: launcher, rendezvous and collectives only",
                              "collective_backend": dist.get_backend() if dist.is_initialized() else None,
                              "max_over_ranks_check": t}), flush=True)
        if dist.is_initialized():
            dist.destroy_process_group()
        return
    torch.cuda.set_device(gpu)
    eng = rxg.Engine(device=gpu)
    stream = None  # the engine's own stream

    seed = shard_seed(0x5EED0001, rank)
    if args.scaling == "strong":  # fixed total, contiguous shares (SURVEY.md 8(d) "Scaling")
        frames = args.total_frames // world + (1 if rank < args.total_frames % world else 0)
    else:
        frames = args.frames
    wl = Workload(eng, args.workload, frames, seed, args.rec)
    tcb, live = rxg.synthetic_tcb_table(wl.flows)
    eng.tcb_load(tcb, live)
    eng.tcb_sync()

    elapsed, region_ms = time_region(eng, wl, args.steps, args.warmup, device, stream)
    cnt = eng.counters()
    elapsed_max = max_over_ranks(elapsed, device)
    merged = merge_counters(cnt, device)
    # per-launch event pairs, a separate pass after the timed region (distribution only)
    _, kern_ms = time_workload(eng, wl, args.steps, 2, device, stream)

    total_frames = int(sum_over_ranks(wl.n, device)) * args.steps
    total_bytes = int(sum_over_ranks(wl.bytes_per_batch, device)) * args.steps
    gbs = total_bytes / elapsed_max / 1e9
    mpps = total_frames / elapsed_max / 1e6
    # the kernel's average launch duration: the timed region's event time / launches
    k_avg_s = region_ms / args.steps / 1e3
    k_med_s = float(np.median(kern_ms)) / 1e3
    # every rank's mean kernel time; the roofline is quoted on the slowest GPU
    k_max_s = max_over_ranks(k_avg_s, device)
    k_min_s = min_over_ranks(k_avg_s, device)
    achieved = wl.bytes_per_batch / k_max_s / 1e9
    C = {name: int(merged[i]) for i, name in enumerate(rxg.COUNTERS)}
    checks_ok = (C["rx"] == total_frames and C["bytes"] == total_bytes
                 and C["ip_cksum_bad"] == 0 and C["tcp_cksum_bad"] == 0
                 and C["dispatch"] == total_frames and C["tcb_hit_exact"] == total_frames)

    legs = {}
    if not args.no_legs:
        # the headline workload with the other record kind (16 <-> 8 bytes), right after the
        # headline timing so that both see the same clocks
        other = rxg.REC16 if args.rec == rxg.REC8 else rxg.REC8
        ow = Workload(eng, args.workload, frames, seed, other)
        _, ro = time_region(eng, ow, args.steps, args.warmup, device, stream)
        ka = max_over_ranks(ro / args.steps / 1e3, device)
        legs[f"{args.workload}_rec{other}"] = {"kernel_us": round(ka * 1e6, 2),
                                               "roofline_frac": round(ow.bytes_per_batch / ka / 1e9 / HBM_PEAK_GBS, 4)}
        ow.free()
        for name, strided in (("c2_64B_1flow", False), ("c2_64B_1flow_strided", True), ("c4_imix_64Kflows", False)):
            wname = name.replace("_strided", "")
            if wname == args.workload:
                continue
            lw = Workload(eng, wname, frames, seed + 99, args.rec)
            t2, l2 = rxg.synthetic_tcb_table(lw.flows)
            eng.tcb_load(t2, l2)
            e2, r2 = time_region(eng, lw, args.steps, args.warmup, device, stream, strided)
            e2 = max_over_ranks(e2, device)
            c2 = merge_counters(eng.counters(), device)
            ka = r2 / args.steps / 1e3
            _, k2 = time_workload(eng, lw, args.steps, 2, device, stream, strided)
            ln = int(sum_over_ranks(lw.n, device)) * args.steps
            lb = int(sum_over_ranks(lw.bytes_per_batch, device)) * args.steps
            legs[name] = {
                "mpps": round(ln / e2 / 1e6, 2),
                "gbs": round(lb / e2 / 1e9, 2),
                "kernel_us": round(ka * 1e6, 2),
                "kernel_us_per_launch_pairs_median": round(float(np.median(k2)) * 1e3, 2),
                "roofline_frac": round(lw.bytes_per_batch / ka / 1e9 / HBM_PEAK_GBS, 4),
                "working_set_GiB": round(lw.copies * (lw.batches[0]["arena_bytes"]) / 2**30, 3),
                "counters_ok": bool(int(c2[0]) == ln
                                    and int(c2[7]) == 0 and int(c2[8]) == 0),
                "descriptors": "fixed stride (no off64[])" if strided else "off64[] + len[]",
                "traffic_bytes_per_launch": traffic_of(name, lw.n, args.rec)[0],
                "algorithmic_bytes_per_launch": lw.bytes_per_batch,
            }
            lw.free()
        legs["c2_64B_1flow_multiburst"] = multiburst_leg(eng, max(5, args.steps // 5), 2, device, seed,
                                                         rec=args.rec)
        legs["c2_64B_1flow_multiburst_strided"] = multiburst_leg(eng, max(5, args.steps // 5), 2, device, seed,
                                                                 rec=args.rec, strided=True)
        # the other record kind on the same ring
        legs[f"c2_64B_1flow_multiburst_rec{other}"] = multiburst_leg(eng, max(5, args.steps // 5), 2, device,
                                                                     seed, rec=other)
        eng.tcb_load(tcb, live)  # the headline's table again (the legs above loaded theirs)
        eng.tcb_sync()
        legs["payload_gather"] = payload_leg(eng, wl, args.steps, 2)
        legs["c3_rx_payload_fused"] = fused_leg(eng, wl, args.steps, 2)
        two = legs["payload_gather"]["kernels_us"] + (region_ms / args.steps * 1e3)
        legs["c3_rx_payload_fused"]["two_pass_us"] = round(two, 2)  # rx_burst_dev + payload_gather_dev
        legs["c3_rx_payload_by_reference"] = fused_leg(eng, wl, args.steps, 2, by_reference=True)
        legs["tx_generate_dev"] = tx_leg(eng, wl, args.steps, 2)
        legs["c3_copy_inclusive"] = copy_inclusive_leg(eng, wl, max(3, args.steps // 4), 1, device)
        legs["c5_bidir_copy_inclusive"] = c5_leg(eng, frames, max(3, args.steps // 4), 1, device,
                                                 seed)
        if rank == 0:  # bounded: SOLO_BUDGET_S (the others wait at the barrier below)
            deadline = time.perf_counter() + min(SOLO_BUDGET_S, args.pg_timeout / 3)
            legs["replay_churn"] = replay_churn_leg(deadline)
            legs["small_burst_latency"] = small_burst_leg(gpu)
        eng.tcb_load(tcb, live)

    # The reference rx path is one lcore (main.c:366-369): its baseline is a host figure,
    # independent of N, timed by rank 0 after the timed region of the N = 1 run only (the
    # driver's N > 1 lines carry null; the other ranks would only wait at the barrier).
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu:
        cores = args.cpu_cores or host_cpus()["usable"]
        cpu = cpu_baseline(eng, wl, seconds=args.cpu_seconds, cores=cores)
    barrier(device)

    traffic, traffic_src = traffic_of(args.workload, wl.n, args.rec)
    prov = rxg.build_provenance()
    tprov = traffic_provenance(traffic_src, prov["build"])
    # every traffic file the line's legs cite, against the same build
    leg_files = sorted({tf for (_, _, r), tf in TRAFFIC_FILES.items() if r == args.rec})
    stale = [tf for tf in leg_files if not traffic_provenance(tf, prov["build"])["traffic_matches_build"]]

    if rank == 0:
        line = {
            "metric": METRIC,
            "value": round(gbs, 2),
            "unit": "GB/s",
            "mpps": round(mpps, 2),
            "n_gpus": world,
            "ranks": ranks,
            "devices": devices,
            "distinct_devices": len({d.get("uuid", d["device"]) for d in devices}),
            "collective_backend": dist.get_backend() if dist.is_initialized() else None,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed_max / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": args.scaling,
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic (device-generated Eth/IPv4/TCP frames, valid checksums, "
                    "SURVEY.md 8(d))",
            "config": {"workload": args.workload, "frames_per_gpu": wl.n,
                       "frame_len": wl.frame_len or "imix", "flows": wl.flows,
                       "tcbs": wl.flows + 1, "record_bytes": args.rec,
                       "record_kind": {8: "RXG_REC8", 16: "RXG_REC16", 48: "RXG_REC48"}[args.rec] +
                       " (record writes are not in the roofline's algorithmic bytes; the REC16 form is "
                       "legs.c3_1500B_1Kflows_rec16)",
                       "bytes_per_gpu_step": wl.bytes_per_batch,
                       "parallelism": f"dp{world} (independent batches, replicated TCB mirror)"},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                         "traffic": traffic,
                         "traffic_source": traffic_src,
                         # the traffic file's counted build against the library measured here
                         "traffic_src": tprov["traffic_src"],
                         "traffic_matches_build": tprov["traffic_matches_build"],
                         "leg_traffic_files": len(leg_files), "leg_traffic_files_stale": stale,
                         "kernel_us": round(k_max_s * 1e6, 2),
                         "kernel_us_per_launch_pairs_rank0_median": round(k_med_s * 1e6, 2),
                         "kernel_us_min_over_ranks": round(k_min_s * 1e6, 2),
                         "kernel_us_max_over_ranks": round(k_max_s * 1e6, 2),
                         "kernel_timing": "one HIP event pair on the launch stream around the timed "
                                          "region's back-to-back launches, / launches (the dispatch gap "
                                          "between launches included); max over ranks.  Per-launch "
                                          "event pairs (a separate pass): kernel_us_per_launch_pairs_*",
                         "algorithmic_bytes_per_launch": wl.bytes_per_batch},
            "cpu_baseline": cpu,
            "counters_ok": bool(checks_ok),
            "counters": C,
            "legs": legs,
            **prov,  # build (src= hash, rev=), lib, source_hash, build_matches_tree
            "pg_timeout_s": args.pg_timeout if dist.is_initialized() else None,
        }
        print(json.dumps(line), flush=True)

    wl.free()
    eng.close()
    if dist.is_initialized():
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
