"""GPU: the burst and its payload hand-off fused in one pass over the frames
(rxg_rx_burst_payload_dev; SURVEY.md §8(a) + §8(f) row 4).

Checked against the oracle (oracle.rx_batch, oracle/payload.py): the records and counters
are those of rxg_rx_burst_dev; the messages are those of rxg_payload_gather_dev (same frames,
len, flags; oracle/payload.slots gives their arena offsets in the pool's geometry); every
message's bytes are its payload; every byte the kernel writes is the pool's own byte at the
same offset, and only the 64-byte lines holding a payload are written (a sentinel arena
shows the rest untouched).  At the BASELINE C3 / C4 sizes through size-independent
properties, and end to end through the C1 stack (burst + replay with PushData taking the
fused payloads) against the reference's sequential loop."""
import random

import numpy as np
import pytest

import c1_stack as c1
import oracle
import pktgen
import rxg
from oracle import payload as opl

pytestmark = pytest.mark.gpu

SENTINEL = 0xA5


def _written_lines(nbytes, exp_msgs):
    """Byte mask of the pool lines the fused kernel writes: each candidate's payload lines."""
    mask = np.zeros(nbytes, dtype=bool)
    for m in exp_msgs:
        if m["len"]:
            start = int(m["arena_off"])
            lo, hi = start // 64, (start + int(m["len"]) - 1) // 64
            mask[lo * 64:(hi + 1) * 64] = True
    return mask


def check_fused(engine, frames, rows, rec_kind=rxg.REC16):
    tcb, live = pktgen.table_arrays(rows)
    engine.tcb_load(tcb, live)
    engine.arp_disable()
    engine.counters_reset()
    recs, parena, msgs, (arena, off, lens) = engine.rx_burst_payload(frames, rec_kind, arena_fill=SENTINEL)
    cnt = engine.counters()
    exp, ecnt = oracle.rx_batch(arena, off, lens, tcb, live)
    if rec_kind == rxg.REC48:
        assert recs.tobytes() == exp.tobytes()
    elif rec_kind == rxg.REC16:
        assert recs.tobytes() == exp["c"].tobytes()
    else:
        assert recs.tobytes() == rxg.rec8_pack(exp["c"]).tobytes()
    assert np.array_equal(cnt, ecnt)
    e_msgs, pays = opl.slots(frames, exp["c"], off)
    for name in ("arena_off", "len", "flags"):
        bad = np.nonzero(msgs[name] != e_msgs[name])[0]
        assert len(bad) == 0, f"msgs.{name} differs at {len(bad)} frames, first {bad[:1]}"
    # the same frames, lengths and flags as the gather's messages
    g_msgs = opl.gather(frames, exp["c"], 1 << 40)[0]
    assert np.array_equal(g_msgs["len"], msgs["len"]) and np.array_equal(g_msgs["flags"], msgs["flags"])
    for i, p in enumerate(pays):
        if p is not None:
            o = int(msgs[i]["arena_off"])
            assert parena[o:o + len(p)].tobytes() == p, f"frame {i}: payload bytes differ"
    mask = _written_lines(len(parena), e_msgs)
    assert np.array_equal(parena[mask], arena[:len(parena)][mask]), "a written byte is not the pool's"
    assert (parena[~mask] == SENTINEL).all(), "a line holding no payload was written"
    return e_msgs


@pytest.mark.parametrize("seed,rec_kind", [(3, rxg.REC16), (4, rxg.REC8), (5, rxg.REC48)])
def test_fused_edge_set(engine, seed, rec_kind):
    rows, frames = pktgen.parity_set(seed, 3000)
    msgs = check_fused(engine, frames, rows, rec_kind)
    got = msgs["flags"] & opl.PM_GATHERED
    assert got.sum() > 500 and (msgs["flags"] & opl.PM_REF_OVERSIZE).sum() > 10


def test_fused_every_payload_length_and_offset(engine):
    """Each payload length 1..200, 990..1010 and a few jumbo ones (the >2 KiB class copies
    its lines separately), data_off 5..15."""
    dst = pktgen.ip4(192, 168, 78, 2)
    rows = [(80, 1024, pktgen.raw_of_host(dst), pktgen.ip4(10, 0, 0, 1), 4)]
    rng = random.Random(9)
    frames = []
    for L in list(range(1, 201)) + list(range(990, 1011)) + [1446, 1500, 2000, 2100, 4000, 9000]:
        for doff in (5, 6, 8, 11, 15):
            frames.append(pktgen.frame(sport=1024, doff=doff, payload=rng.randbytes(L),
                                       tcp_opts=rng.randbytes((doff - 5) * 4)))
    msgs = check_fused(engine, frames, rows)
    assert (msgs["flags"] & opl.PM_GATHERED).all()


def test_fused_matches_burst_then_gather(engine):
    """rxg_rx_burst_payload_dev vs rxg_rx_burst_dev + rxg_payload_gather_dev on the same device
    batch: same records, same counters, every message the same bytes."""
    rows, frames = pktgen.parity_set(8, 4000)
    tcb, live = pktgen.table_arrays(rows)
    engine.tcb_load(tcb, live)
    engine.arp_disable()
    engine.counters_reset()
    recs_f, parena, msgs_f, _ = engine.rx_burst_payload(frames, rxg.REC16)
    cnt_f = engine.counters()
    engine.counters_reset()
    recs_g = engine.rx_burst(frames, rxg.REC16)
    cnt_g = engine.counters()
    g_arena, g_msgs, _ = engine.payload_gather(len(frames), 4096 + 2048 * len(frames))
    assert recs_f.tobytes() == recs_g.tobytes() and np.array_equal(cnt_f, cnt_g)
    assert np.array_equal(msgs_f["len"], g_msgs["len"]) and np.array_equal(msgs_f["flags"], g_msgs["flags"])
    for i in np.nonzero(g_msgs["len"])[0]:
        L = int(g_msgs[i]["len"])
        a, b = int(msgs_f[i]["arena_off"]), int(g_msgs[i]["arena_off"])
        assert parena[a:a + L].tobytes() == g_arena[b:b + L].tobytes()


def _fused_full(engine, n, flows, seed, mix, len_a=1500, by_reference=False):
    b = engine.synth(n=n, nflows=flows, len_a=len_a, mix=mix, seed=seed)
    tcb, live = rxg.synthetic_tcb_table(flows)
    engine.tcb_load(tcb, live)
    engine.tcb_sync()
    nb = b["arena_bytes"]
    recs, msgs = engine.alloc(n * 8), engine.alloc(n * 16)
    parena = None
    if not by_reference:
        parena = engine.alloc(nb)
        parena.upload(np.full(nb, SENTINEL, dtype=np.uint8))
    engine.counters_reset()
    engine.rx_burst_payload_dev(b["arena"].ptr, b["off64"].ptr, b["len"].ptr, n, recs.ptr,
                                parena.ptr if parena else None, msgs.ptr, rxg.REC8)
    engine.sync()
    return b, recs, msgs, parena


def test_fused_c3_full_size_property(engine):
    """BASELINE C3 (2^20 x 1500 B, 1000 flows): every frame DISPATCH, both checksums valid,
    every payload handed off (1 446 bytes at 64 * off64 + 54), the arena equal to the pool in
    every frame's 24 lines (the whole slot: the payload spans lines 0..23)."""
    n, flows = 1 << 20, 1000
    b, recs, msgs, parena = _fused_full(engine, n, flows, 0x5EED0001, 0)
    c = dict(zip(rxg.COUNTERS, engine.counters().tolist()))
    assert c["rx"] == n and c["dispatch"] == n and c["tcb_hit_exact"] == n
    assert c["ip_cksum_bad"] == 0 and c["tcp_cksum_bad"] == 0
    r = rxg.rec8_expand(recs.download(rxg.REC8_DTYPE, n))
    assert (r["verdict"] == rxg.V_DISPATCH).all() and (r["datalen"] == 1446).all()
    m = msgs.download(rxg.PAYLOAD_MSG_DTYPE, n)
    off = b["off64"].download(np.uint32, n).astype(np.uint64)
    assert (m["len"] == 1446).all() and (m["arena_off"] == off * 64 + 54).all()
    assert (m["flags"] == (rxg.PM_GATHERED | rxg.PM_REF_OVERSIZE)).all()
    nb = b["arena_bytes"]
    for c0 in range(0, nb, 1 << 28):  # in pieces (host memory)
        k = min(1 << 28, nb - c0)
        fr = b["arena"].download(np.uint8, k, offset_bytes=c0)
        pa = parena.download(np.uint8, k, offset_bytes=c0)
        assert np.array_equal(fr, pa), f"arena differs from the pool in [{c0}, {c0 + k})"
    for d in list(b.values()) + [recs, msgs, parena]:
        if isinstance(d, rxg.DevArray):
            d.free()


def test_fused_c4_imix_full_size_property(engine):
    """BASELINE C4 batch (2^20 IMIX 64/576/1500, 64 K flows): every payload handed off at its
    frame's offset (64 * off64 + 54, length len - 54), and the arena equal to the pool over
    each frame's lines (64 B: its one line; 576 B: 9 lines; 1 500 B: 24)."""
    n, flows = 1 << 20, 65536
    b, recs, msgs, parena = _fused_full(engine, n, flows, 0x5EED0004, 1)
    c = dict(zip(rxg.COUNTERS, engine.counters().tolist()))
    assert c["rx"] == n and c["dispatch"] == n and c["tcp_cksum_bad"] == 0
    m = msgs.download(rxg.PAYLOAD_MSG_DTYPE, n)
    off = b["off64"].download(np.uint32, n).astype(np.uint64)
    lens = b["len"].download(np.uint16, n).astype(np.uint64)
    assert (m["len"] == lens - 54).all() and (m["arena_off"] == off * 64 + 54).all()
    assert ((m["flags"] & rxg.PM_GATHERED) != 0).all()
    nb = b["arena_bytes"]
    fr = b["arena"].download(np.uint8, nb).reshape(-1, 64)
    pa = parena.download(np.uint8, nb).reshape(-1, 64)
    # the lines of every frame (each frame's payload spans all of them), and no other line
    cnt = (lens.astype(np.int64) + 63) // 64
    first = off.astype(np.int64)
    line = np.repeat(first - np.concatenate([[0], np.cumsum(cnt)[:-1]]), cnt) + np.arange(int(cnt.sum()))
    written = np.zeros(len(fr), dtype=bool)
    written[line] = True
    assert np.array_equal(fr[written], pa[written]), "a payload line differs from the pool"
    assert (pa[~written] == SENTINEL).all(), "a line outside every frame was written"
    for d in list(b.values()) + [recs, msgs, parena]:
        if isinstance(d, rxg.DevArray):
            d.free()


@pytest.mark.parametrize("seed", [1, 2])
def test_fused_multiflow_exchange_equals_reference(engine, seed):
    """End to end: burst + hand-off in one pass, then the replay, PushData taking the fused
    payloads (rxg_payload_take): every socket-ring message equals the reference's."""
    from test_gpu_payload import multiflow_bursts
    bursts = multiflow_bursts(seed)
    ref = c1.drive_cpu(bursts)
    got = c1.drive_rxg(engine, bursts, fused=True)
    assert got.rings == ref.rings
    assert got.log == ref.log and got.rows == ref.rows
    assert got.sent == ref.sent
    assert got.taken == ref.eligible and got.eligible == 0 and got.taken > 200


@pytest.mark.parametrize("rec_kind", [rxg.REC16, rxg.REC8])
def test_fused_by_reference(engine, rec_kind):
    """arena NULL: nothing copied; the same records, counters and messages, each message
    naming its payload in the frame pool itself (the payload bytes read from there)."""
    rows, frames = pktgen.parity_set(12, 3000)
    tcb, live = pktgen.table_arrays(rows)
    engine.tcb_load(tcb, live)
    engine.arp_disable()
    engine.counters_reset()
    recs, pool, msgs, (arena, off, lens) = engine.rx_burst_payload(frames, rec_kind, by_reference=True)
    cnt = engine.counters()
    exp, ecnt = oracle.rx_batch(arena, off, lens, tcb, live)
    want = exp["c"].tobytes() if rec_kind == rxg.REC16 else rxg.rec8_pack(exp["c"]).tobytes()
    assert recs.tobytes() == want and np.array_equal(cnt, ecnt)
    assert pool.tobytes() == arena.tobytes()  # the pool itself, untouched
    e_msgs, pays = opl.slots(frames, exp["c"], off)
    assert msgs.tobytes() == e_msgs.tobytes()
    for i, p in enumerate(pays):
        if p is not None:
            o = int(msgs[i]["arena_off"])
            assert pool[o:o + len(p)].tobytes() == p


def test_fused_by_reference_multiflow_exchange(engine):
    """The C1 stack end to end with the hand-off by reference: PushData takes every eligible
    payload from the pool, and the socket rings equal the reference's."""
    from test_gpu_payload import multiflow_bursts
    bursts = multiflow_bursts(3)
    ref = c1.drive_cpu(bursts)
    got = c1.drive_rxg(engine, bursts, fused=True, by_reference=True)
    assert got.rings == ref.rings and got.log == ref.log and got.sent == ref.sent
    assert got.taken == ref.eligible and got.taken > 200


@pytest.mark.parametrize("len_a,by_ref", [(1500, False), (64, False), (576, False), (1500, True)])
def test_fused_strided_equals_list_form(engine, len_a, by_ref):
    """rxg_rx_burst_strided_payload_dev (frame i at slot slot0 + i * stride64, no off64[]) against
    rxg_rx_burst_payload_dev over the same frames through their offset list: same records,
    counters, messages and payload lines; a burst starting mid-pool (slot0 > 0)."""
    n, flows = 20000, 500
    b = engine.synth(n=n, nflows=flows, len_a=len_a, seed=0x5EED00AA)
    tcb, live = rxg.synthetic_tcb_table(flows)
    engine.tcb_load(tcb, live)
    engine.tcb_sync()
    stride = (len_a + 63) // 64
    k0 = 3000  # the burst: frames k0 .. n-1
    m = n - k0
    nb = b["arena_bytes"]
    outs = []
    for form in ("list", "stride"):
        recs, msgs = engine.alloc(m * 16), engine.alloc(m * 16)
        pa = None if by_ref else engine.alloc(nb)
        if pa is not None:
            pa.upload(np.full(nb, SENTINEL, dtype=np.uint8))
        engine.counters_reset()
        if form == "list":
            engine.rx_burst_payload_dev(b["arena"].ptr, b["off64"].ptr + 4 * k0, b["len"].ptr + 2 * k0, m, recs.ptr,
                                        pa.ptr if pa else None, msgs.ptr, rxg.REC16)
        else:
            engine.rx_burst_strided_payload_dev(b["arena"].ptr, stride, k0 * stride, b["len"].ptr + 2 * k0, m,
                                                recs.ptr, pa.ptr if pa else None, msgs.ptr, rxg.REC16)
        engine.sync()
        outs.append((recs.download(np.uint8, m * 16).tobytes(), engine.counters().tolist(),
                     msgs.download(rxg.PAYLOAD_MSG_DTYPE, m), pa.download(np.uint8, nb).tobytes() if pa else None))
        for d in (recs, msgs, pa):
            if d is not None:
                d.free()
    (r1, c1_, m1, a1), (r2, c2_, m2, a2) = outs
    assert r1 == r2 and c1_ == c2_ and m1.tobytes() == m2.tobytes() and a1 == a2
    off = b["off64"].download(np.uint32, n)[k0:].astype(np.uint64)
    assert (m1["arena_off"] == off * 64 + 54).all() and (m1["len"] == len_a - 54).all()
    for d in b.values():
        if isinstance(d, rxg.DevArray):
            d.free()


@pytest.mark.parametrize("mix", [0, 1])
def test_fused_by_reference_full_size_property(engine, mix):
    """The by-reference form at the BASELINE C3 / C4 sizes (2^20 frames: 5-6 slices per wave on
    the occupancy grid, records and messages out of the ring at each wave's end): the
    records and counters equal the copy form's, every message names its payload in the pool
    (64 * off64 + 54, length len - 54), and the pool is untouched."""
    n, flows, seed = 1 << 20, (1000, 65536)[mix], (0x5EED0001, 0x5EED0004)[mix]
    b, recs, msgs, _ = _fused_full(engine, n, flows, seed, mix, by_reference=True)
    cnt_ref = engine.counters()
    r_ref = recs.download(np.uint8, n * 8)
    m = msgs.download(rxg.PAYLOAD_MSG_DTYPE, n)
    nb = b["arena_bytes"]
    pool_sum = int(b["arena"].download(np.uint64, nb // 8).sum())  # (wrapping word sum)
    off = b["off64"].download(np.uint32, n).astype(np.uint64)
    lens = b["len"].download(np.uint16, n).astype(np.uint64)
    assert (m["len"] == lens - 54).all() and (m["arena_off"] == off * 64 + 54).all()
    want_flags = rxg.PM_GATHERED | np.where(lens - 54 >= 1000, rxg.PM_REF_OVERSIZE, 0)
    assert (m["flags"] == want_flags).all()
    # the copy form over the same batch: the same records and counters
    parena = engine.alloc(nb)
    engine.counters_reset()
    engine.rx_burst_payload_dev(b["arena"].ptr, b["off64"].ptr, b["len"].ptr, n, recs.ptr, parena.ptr, msgs.ptr,
                                rxg.REC8)
    engine.sync()
    assert np.array_equal(engine.counters(), cnt_ref)
    assert recs.download(np.uint8, n * 8).tobytes() == r_ref.tobytes()
    assert int(b["arena"].download(np.uint64, nb // 8).sum()) == pool_sum
    for d in list(b.values()) + [recs, msgs, parena]:
        if isinstance(d, rxg.DevArray):
            d.free()
