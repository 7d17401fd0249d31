"""GPU: latency mode (include/rxg.h rxg_server_*).  A persistent kernel serves bursts posted
through a mailbox (device memory the host writes through the BAR, or coherent host memory:
both placements are tested); its records, counters and replay must equal the launched path's
and the oracle's, burst after burst (fresh frame content each time: no stale reads of the
staging), across mirror writes, idle exits and restarts."""
import random
import time

import numpy as np
import pytest

import oracle
import pktgen
import rxg
import test_gpu_replay
from test_gpu_parity import assert_records_equal

pytestmark = pytest.mark.gpu


@pytest.fixture
def srv_engine():
    eng = rxg.Engine(device=0, max_batch=1 << 16, max_bytes=64 << 20)
    yield eng
    eng.close()


# rxg_server_config.flags: 0 = placed by the device (device memory on a large-BAR GPU),
# SRV_HOST_STAGING = coherent host memory
PLACEMENTS = [0, rxg.SRV_HOST_STAGING, rxg.SRV_HOST_MAILBOX]


def test_server_placement_reported(srv_engine):
    """flags 0 puts the mailbox and staging in device memory when the GPU exposes it to the
    host (large BAR, as on the MI355X boxes); RXG_SRV_HOST_STAGING keeps them in host memory."""
    eng = srv_engine
    assert eng.server_placement() == rxg.SRV_NONE
    eng.server_start(rxg.REC8, max_frames=64, flags=rxg.SRV_HOST_STAGING)
    assert eng.server_placement() == rxg.SRV_HOST
    eng.server_start(rxg.REC8, max_frames=64)
    assert eng.server_placement() in (rxg.SRV_DEVICE, rxg.SRV_HOST)
    eng.server_stop()
    assert eng.server_placement() == rxg.SRV_NONE


def _upload(eng, arena, off, lens):
    return eng.to_device(arena), eng.to_device(off.astype(np.uint32)), eng.to_device(lens.astype(np.uint16))


@pytest.mark.parametrize("flags", PLACEMENTS)
@pytest.mark.parametrize("blocks", [1, 3])
def test_server_bursts_equal_launched(srv_engine, blocks, flags):
    """Sub-bursts of every shape (1 .. 4096 frames, partial slices) of one device batch: the
    served records equal one launched burst's, byte for byte, and so do the counters."""
    eng = srv_engine
    rows, frames = pktgen.parity_set(seed=71 + blocks, n=6000)
    arena, off, lens = pktgen.pack_arena(frames)
    tcb, live = pktgen.table_arrays(rows)
    eng.tcb_load(tcb, live)
    n = len(lens)
    d_arena, d_off, d_len = _upload(eng, arena, off, lens)
    ref = eng.alloc(n * 16)
    out = eng.alloc(n * 16)
    try:
        eng.counters_reset()
        eng.rx_burst_dev(d_arena.ptr, d_off.ptr, d_len.ptr, n, ref.ptr, rxg.REC16)
        eng.sync()
        exp_cnt = eng.counters()
        exp = ref.download(np.uint8, n * 16)
        eng.server_start(rxg.REC16, blocks=blocks, max_frames=4096, flags=flags)
        assert eng.server_active()
        eng.counters_reset()
        i = 0
        for k in [1, 32, 63, 64, 65, 100, 255, 1000, 4096, 3, 32, 32, 31, 257] * 2:
            k = min(k, n - i)
            if k == 0:
                break
            eng.server_burst_dev(d_arena.ptr, d_off.ptr + 4 * i, d_len.ptr + 2 * i, k, out.ptr + 16 * i, rxg.REC16)
            i += k
        got = out.download(np.uint8, i * 16)
        assert got.tobytes() == exp[: i * 16].tobytes()
        if i == n:
            assert eng.counters().tolist() == exp_cnt.tolist()
        eng.server_stop()
        assert not eng.server_active()
    finally:
        for d in (d_arena, d_off, d_len, ref, out):
            d.free()


@pytest.mark.parametrize("flags", PLACEMENTS)
@pytest.mark.parametrize("rec", [rxg.REC8, rxg.REC16, rxg.REC48])
def test_server_host_bursts_equal_launched_and_oracle(srv_engine, rec, flags):
    """rxg_rx_burst through the server: 200 consecutive bursts of the reference's size class
    (1..64 frames, fresh content every burst) equal the same bursts launched, and (REC48,
    every field) the oracle."""
    eng = srv_engine
    rows, frames = pktgen.parity_set(seed=90 + rec, n=4000)
    tcb, live = pktgen.table_arrays(rows)
    eng.tcb_load(tcb, live)
    rng = np.random.default_rng(rec)
    bursts, i = [], 0
    for _ in range(200):
        k = int(rng.integers(1, 65))
        bursts.append(frames[i:i + k])
        i += k
    eng.server_start(rec, max_frames=256, flags=flags)
    try:
        served = [eng.rx_burst(b, rec) for b in bursts]
    finally:
        eng.server_stop()
    for b, got in zip(bursts, served):
        assert eng.rx_burst(b, rec).tobytes() == got.tobytes()
        if rec == rxg.REC48:
            arena, off, lens = pktgen.pack_arena(b)
            exp, _ = oracle.rx_batch(arena, off, lens, tcb, live)
            assert_records_equal(got, exp, b)


@pytest.mark.parametrize("flags", PLACEMENTS)
@pytest.mark.parametrize("blocks", [1, 3])
def test_server_sees_mirror_writes(srv_engine, blocks, flags):
    """tcbs[] writes between served bursts (upsert, remove, set_state) are on the device
    before the next burst reads the table: each served burst equals the oracle on the table
    as it stands."""
    eng = srv_engine
    rows, frames = pktgen.parity_set(seed=5, n=1024, nflows=64)
    tcb, live = pktgen.table_arrays(rows)
    eng.tcb_load(tcb, live)
    eng.server_start(rxg.REC48, blocks=blocks, max_frames=512, flags=flags)
    rng = np.random.default_rng(5 + blocks)
    try:
        for step in range(30):
            idx = int(rng.integers(1, len(tcb)))
            if step % 3 == 0:
                live[idx] = 0
                eng.tcb_remove(idx)
            elif step % 3 == 1 and live[idx]:
                st = rxg.TCP_ESTABLISHED if tcb["state"][idx] != rxg.TCP_ESTABLISHED else rxg.LISTENING
                tcb["state"][idx] = st
                eng.tcb_set_state(idx, st)
            else:
                live[idx] = 1
                t = tcb[idx]
                eng.tcb_upsert(idx, int(t["dport"]), int(t["sport"]), int(t["ipv4_dst"]), int(t["ipv4_src"]),
                               int(t["state"]), int(t["identifier"]))
            fr = frames[step * 32: step * 32 + 32]
            got = eng.rx_burst(fr, rxg.REC48)
            arena, off, lens = pktgen.pack_arena(fr)
            exp, _ = oracle.rx_batch(arena, off, lens, tcb, live)
            assert_records_equal(got, exp, fr)
    finally:
        eng.server_stop()


@pytest.mark.parametrize("flags", PLACEMENTS)
def test_server_idle_exit_and_relaunch(srv_engine, flags):
    """A server idle for longer than idle_ms exits; the next burst relaunches it.  Stop and
    start again; a context closed with a running server stops it."""
    eng = srv_engine
    rows, frames = pktgen.parity_set(seed=11, n=256)
    tcb, live = pktgen.table_arrays(rows)
    eng.tcb_load(tcb, live)
    arena, off, lens = pktgen.pack_arena(frames[:40])
    exp = eng.rx_arena(arena, off, lens, rxg.REC16)
    eng.server_start(rxg.REC16, max_frames=64, idle_ms=30, flags=flags)
    for _ in range(3):
        assert eng.rx_burst(frames[:40], rxg.REC16).tobytes() == exp.tobytes()
        time.sleep(0.15)  # the kernel exits idle
        assert eng.rx_burst(frames[:40], rxg.REC16).tobytes() == exp.tobytes()
    eng.server_stop()
    eng.server_start(rxg.REC16, max_frames=64)
    assert eng.rx_burst(frames[:40], rxg.REC16).tobytes() == exp.tobytes()
    # too large for the server: launched as before
    assert eng.rx_burst(frames[:200], rxg.REC16).shape[0] == 200
    other = rxg.Engine(device=0, max_batch=256, max_bytes=1 << 20)
    other.server_start(rxg.REC8, max_frames=64)
    other.close()  # stops its server


def test_server_rejects_bad_requests(srv_engine):
    eng = srv_engine
    lib = rxg.load_library()
    import ctypes as C
    b = rxg.DevBatch(None, None, None, 1, rxg.REC8, None)
    assert lib.rxg_server_burst_dev(eng.ctx, C.byref(b)) < 0  # no server
    eng.server_start(rxg.REC8, max_frames=64)
    try:
        b = rxg.DevBatch(None, None, None, 65, rxg.REC8, None)
        assert lib.rxg_server_burst_dev(eng.ctx, C.byref(b)) < 0  # too many
        b = rxg.DevBatch(None, None, None, 1, rxg.REC16, None)
        assert lib.rxg_server_burst_dev(eng.ctx, C.byref(b)) < 0  # wrong kind
        b = rxg.DevBatch(None, None, None, 1, rxg.REC8, None)
        assert lib.rxg_server_burst_dev(eng.ctx, C.byref(b)) < 0  # NULL pointers
        cfg = rxg.ServerConfig(7, 1, 64, 0, 0, 0)
        assert lib.rxg_server_start(eng.ctx, C.byref(cfg)) < 0
    finally:
        eng.server_stop()


@pytest.mark.parametrize("seed,on_device,flags", [(1, False, 0), (2, False, rxg.SRV_HOST_STAGING), (3, True, 0),
                                                  (4, True, rxg.SRV_HOST_STAGING)])
def test_server_replay_sequential_equivalence(seed, on_device, flags):
    """The replay test of test_gpu_replay (in-burst SYN/FIN writes re-classified) with the
    burst served instead of launched; on_device: every fix-up a GPU re-classify launch, which
    reads the served burst's frames in the server's staging."""
    eng = rxg.Engine(device=0, max_batch=1 << 16, max_bytes=64 << 20,
                     flags=rxg.CFG_REPLAY_ON_DEVICE if on_device else 0)
    eng.server_start(rxg.REC16, blocks=2, max_frames=4096, flags=flags)
    try:
        test_gpu_replay.run_replay_equivalence(eng, seed)
    finally:
        eng.close()


def test_launched_bursts_beside_a_running_server(srv_engine):
    """Launched bursts (another stream of the same context) run beside the resident server and
    interleave with served ones; every record equals the oracle's."""
    eng = srv_engine
    rows, frames = pktgen.parity_set(seed=21, n=3000)
    arena, off, lens = pktgen.pack_arena(frames)
    tcb, live = pktgen.table_arrays(rows)
    eng.tcb_load(tcb, live)
    exp, _ = oracle.rx_batch(arena, off, lens, tcb, live)
    n = len(lens)
    d_arena, d_off, d_len = _upload(eng, arena, off, lens)
    out = eng.alloc(n * 48)
    eng.server_start(rxg.REC48, blocks=2, max_frames=256)
    try:
        for rep in range(3):
            eng.rx_burst_dev(d_arena.ptr, d_off.ptr, d_len.ptr, n, out.ptr, rxg.REC48)  # launched
            eng.sync()
            assert_records_equal(out.download(np.uint8, n * 48).view(rxg.REC48_DTYPE), exp, frames)
            i = 100 * rep
            got = eng.rx_burst(frames[i:i + 40], rxg.REC48)  # served
            assert_records_equal(got, exp[i:i + 40], frames[i:i + 40])
    finally:
        eng.server_stop()
        for d in (d_arena, d_off, d_len, out):
            d.free()


def _free_all(*objs):
    for o in objs:
        if isinstance(o, dict):
            for v in o.values():
                if isinstance(v, rxg.DevArray):
                    v.free()
        elif o is not None:
            o.free()


def test_server_alternating_participants():
    """64 workgroups serve 2 100 requests whose sizes alternate so that the
    number of participating workgroups P changes every request (32 frames: P = 1, 300: 2,
    4 096: 16, 16 384: 64), so workgroups keep sitting requests out while others run the next
    one.  Every served request's records equal the launched burst's of the same frames, and
    the counters of the whole sequence equal those of the same sequence launched.  (Round 3's
    forwarding let a workgroup that sat out read the next request's words under the old
    request's number.)"""
    eng = rxg.Engine(device=0)
    n = 16384
    dev = eng.synth(n=n, nflows=4096, mix=1, seed=404)
    tcb, live = rxg.synthetic_tcb_table(4096)
    eng.tcb_load(tcb, live)
    ref, out = eng.alloc(n * 8), eng.alloc(n * 8)
    rng = np.random.default_rng(404)
    sizes = [32, 300, 4096, 16384]
    reqs = []
    for j in range(2100):
        k = sizes[j % 4] if j % 7 else sizes[int(rng.integers(0, 4))]
        i = int(rng.integers(0, n - k + 1))
        reqs.append((i, k))
    try:
        eng.rx_burst_dev(dev["arena"].ptr, dev["off64"].ptr, dev["len"].ptr, n, ref.ptr, rxg.REC8)
        eng.sync()
        exp = ref.download(np.uint8, n * 8)
        # the counters of the sequence, launched
        eng.counters_reset()
        for i, k in reqs:
            eng.rx_burst_dev(dev["arena"].ptr, dev["off64"].ptr + 4 * i, dev["len"].ptr + 2 * i, k, out.ptr, rxg.REC8)
        eng.sync()
        exp_cnt = eng.counters()
        eng.server_start(rxg.REC8, blocks=64, max_frames=n)
        eng.counters_reset()
        for j, (i, k) in enumerate(reqs):
            eng.server_burst_dev(dev["arena"].ptr, dev["off64"].ptr + 4 * i, dev["len"].ptr + 2 * i, k,
                                 out.ptr + 8 * i, rxg.REC8)
            if j % 5 == 0 or k == n:  # (every request's records at the end of the loop too)
                got = out.download(np.uint8, k * 8, offset_bytes=8 * i)
                assert got.tobytes() == exp[8 * i: 8 * (i + k)].tobytes(), (j, i, k)
        assert eng.counters().tolist() == exp_cnt.tolist()
        eng.server_stop()
    finally:
        _free_all(dev, ref, out)
        eng.close()


@pytest.mark.parametrize("flags", [0, rxg.SRV_HOST_STAGING])
def test_server_overflow_walks_see_mirror_writes(flags):
    """the overflow walks (tuples and ARP addresses past their first bucket)
    of the resident server read the mirror as it stands after writes made between requests.
    64 K TCBs at the mirror's load (full first buckets are common: ~0.4 % of the probes walk),
    a thousand removals / re-insertions between served bursts (backward-shift deletions move
    tuples across buckets) and ARP addresses learned between them: every served burst equals
    the same burst launched on the same table."""
    eng = rxg.Engine(device=0)
    nflows, n = 65536, 8192
    dev = eng.synth(n=n, nflows=nflows, len_a=64, seed=505, with_flows=True)
    tcb, live = rxg.synthetic_tcb_table(nflows)
    live = live.copy()
    eng.tcb_load(tcb, live)
    srcs = tcb["ipv4_src"][1:]
    eng.arp_load(srcs[: nflows // 2])
    learned = nflows // 2
    ref, out = eng.alloc(n * 16), eng.alloc(n * 16)
    rng = np.random.default_rng(505)
    try:
        eng.server_start(rxg.REC16, blocks=8, max_frames=n, flags=flags)
        for step in range(12):
            for idx in rng.choice(np.arange(1, nflows + 1), size=1000, replace=False):
                idx = int(idx)
                if live[idx]:
                    live[idx] = 0
                    eng.tcb_remove(idx)
                else:
                    live[idx] = 1
                    t = tcb[idx]
                    eng.tcb_upsert(idx, int(t["dport"]), int(t["sport"]), int(t["ipv4_dst"]), int(t["ipv4_src"]),
                                   int(t["state"]), int(t["identifier"]))
            for ip in srcs[learned: learned + 1500]:
                eng.arp_learned(int(ip))
            learned += 1500
            eng.server_burst_dev(dev["arena"].ptr, dev["off64"].ptr, dev["len"].ptr, n, out.ptr, rxg.REC16)
            got = out.download(np.uint8, n * 16)
            eng.rx_burst_dev(dev["arena"].ptr, dev["off64"].ptr, dev["len"].ptr, n, ref.ptr, rxg.REC16)
            eng.sync()
            exp = ref.download(np.uint8, n * 16)
            assert got.tobytes() == exp.tobytes(), step
            r = got.view(rxg.REC16_DTYPE)
            assert (r["flags"] & rxg.F_ARP_LEARN).any() and not (r["flags"] & rxg.F_ARP_LEARN).all()
        eng.server_stop()
    finally:
        _free_all(dev, ref, out)
        eng.close()


@pytest.mark.parametrize("flags", PLACEMENTS)
def test_server_small_bursts_of_every_size_class(srv_engine, flags):
    """Round 4's server forms for a request of one slice (HISTORY.md §9.R4): descriptors
    carried in the mailbox (host bursts of <= 32 frames), the all-small path for a partial
    slice of small frames, and the workgroup's four waves sharing the streaming-class rounds
    of a slice of >= 8 frames.  Bursts of 1..64 frames holding every size class (small, 65-128,
    .., 1 025-1 536, 1 537-2 048, jumbo) or only small frames, each served, launched and (REC48,
    every field) run through the oracle: equal."""
    eng = srv_engine
    rng = random.Random(404)
    rows, flows, _ = pktgen.parity_table(rng, 50)
    tcb, live = pktgen.table_arrays(rows)
    eng.tcb_load(tcb, live)
    sizes = [60, 64, 100, 200, 400, 550, 700, 900, 1500, 2000, 4000, 9000]
    bursts = []
    for k in [1, 2, 7, 8, 9, 12, 31, 32, 33, 63, 64]:
        for small_only in (False, True):
            b = []
            for i in range(k):
                L = rng.choice(sizes[:2]) if small_only else sizes[i % len(sizes)] if i < len(sizes) else rng.choice(sizes)
                src, sport, dport = rng.choice(flows)
                f = pktgen.frame(src_ip=src, sport=sport, dport=dport, payload=rng.randbytes(max(0, L - 54)),
                                 flags=rng.choice([0x02, 0x10, 0x18]))
                b.append(f[:L])
            bursts.append(b)
    eng.server_start(rxg.REC48, blocks=1, max_frames=64, flags=flags)
    try:
        served = [eng.rx_burst(b, rxg.REC48) for b in bursts]
    finally:
        eng.server_stop()
    for b, got in zip(bursts, served):
        assert eng.rx_burst(b, rxg.REC48).tobytes() == got.tobytes(), len(b)
        arena, off, lens = pktgen.pack_arena(b)
        exp, _ = oracle.rx_batch(arena, off, lens, tcb, live)
        assert_records_equal(got, exp, b)
