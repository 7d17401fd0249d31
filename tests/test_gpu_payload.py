"""GPU: the payload hand-off — rxg_payload_gather_dev bit-exact
against oracle/payload.py on the rx edge-case set, at the BASELINE C3 size through a
size-independent property, and end to end: a multi-flow exchange through rxg (burst +
gather + replay, PushData taking gathered payloads) equals the reference's sequential
rx loop + receive window (oracle/window.py) message for message."""
import random

import numpy as np
import pytest

import c1_stack as c1
import oracle
import pktgen
import rxg
from oracle import payload as opl
from oracle import window as ow

pytestmark = pytest.mark.gpu


def check_gather(engine, frames, rows, cap=None, rec_kind=rxg.REC16):
    tcb, live = pktgen.table_arrays(rows)
    engine.tcb_load(tcb, live)
    engine.arp_disable()
    recs = engine.rx_burst(frames, rec_kind)
    arena, off, lens = pktgen.pack_arena(frames)
    exp_recs, _ = oracle.rx_batch(arena, off, lens, tcb, live)
    c16 = recs["c"] if rec_kind == rxg.REC48 else recs
    assert c16.tobytes() == exp_recs["c"].tobytes()
    full = opl.gather(frames, exp_recs["c"], 1 << 40)[2]
    cap = full if cap is None else cap
    e_msgs, e_arena, e_used = opl.gather(frames, exp_recs["c"], cap)
    g_arena, g_msgs, g_used = engine.payload_gather(len(frames), cap)
    assert g_used == e_used == full
    for name in ("arena_off", "len", "flags"):
        bad = np.nonzero(g_msgs[name] != e_msgs[name])[0]
        assert len(bad) == 0, f"msgs.{name} differs at {len(bad)} frames, first {bad[0]}"
    assert g_arena[:len(e_arena)].tobytes() == e_arena.tobytes()
    return e_msgs


@pytest.mark.parametrize("seed", [3, 4])
def test_gather_edge_set(engine, seed):
    rows, frames = pktgen.parity_set(seed, 3000)
    msgs = check_gather(engine, frames, rows)
    got = msgs["flags"] & opl.PM_GATHERED
    assert got.sum() > 500 and (msgs["flags"] & opl.PM_REF_OVERSIZE).sum() > 10


def test_gather_rec48_and_arena_overflow(engine):
    rows, frames = pktgen.parity_set(5, 2000)
    check_gather(engine, frames, rows, rec_kind=rxg.REC48)
    msgs = check_gather(engine, frames, rows, cap=20000)
    assert 0 < (msgs["flags"] & opl.PM_GATHERED).sum() < 200


def test_gather_arena_capacity_sweep(engine):
    """Capacities at, just below and just above message boundaries (the copy is issued
    before the workgroup's arena offset is known, so payloads past the capacity are loaded
    and must not be stored, nor get a message)."""
    rows, frames = pktgen.parity_set(6, 3000)
    tcb, live = pktgen.table_arrays(rows)
    arena, off, lens = pktgen.pack_arena(frames)
    exp_recs, _ = oracle.rx_batch(arena, off, lens, tcb, live)
    msgs, _, full = opl.gather(frames, exp_recs["c"], 1 << 40)
    starts = np.sort(msgs["arena_off"][msgs["len"] > 0])
    assert len(starts) > 500
    caps = {16, full - 16, full}
    for k in (1, len(starts) // 7, len(starts) // 2, len(starts) - 1):
        b = int(starts[k])
        caps |= {b - 1, b, b + 1, b + 16}
    for cap in sorted(c for c in caps if 0 < c <= full):
        m = check_gather(engine, frames, rows, cap=cap)
        got = m["flags"] & opl.PM_GATHERED
        assert (m["arena_off"][got > 0] + m["len"][got > 0] <= cap).all()
        # nothing is written past the capacity: a guard of sentinel bytes after it
        guard = 4096
        da, dm, du = engine.alloc(cap + guard), engine.alloc(len(frames) * 16), engine.alloc(8)
        try:
            da.upload(np.full(cap + guard, 0xA5, dtype=np.uint8))
            engine.payload_gather_dev(da.ptr, cap, dm.ptr, du.ptr)
            engine.sync()
            tail = da.download(np.uint8, guard, offset_bytes=cap)
            assert (tail == 0xA5).all(), f"cap {cap}: the gather wrote past the arena capacity"
        finally:
            for d in (da, dm, du):
                d.free()


def test_gather_every_payload_length_and_offset(engine):
    """Each payload length 1..200 and 990..1010, data_off 5..15 (source alignment)."""
    dst = pktgen.ip4(192, 168, 78, 2)
    rows = [(80, 1024, pktgen.raw_of_host(dst), pktgen.ip4(10, 0, 0, 1), 4)]
    rng = random.Random(9)
    frames = []
    for L in list(range(1, 201)) + list(range(990, 1011)):
        for doff in (5, 6, 8, 11, 15):
            frames.append(pktgen.frame(sport=1024, doff=doff, payload=rng.randbytes(L),
                                       tcp_opts=rng.randbytes((doff - 5) * 4)))
    msgs = check_gather(engine, frames, rows)
    assert (msgs["flags"] & opl.PM_GATHERED).all()


def test_gather_c3_full_size_property(engine):
    """BASELINE C3 (2^20 x 1500 B, 1000 flows): every payload gathered, the arena equals
    the frames' bytes 54..1500, in order, each message padded to 1456 bytes."""
    n, flows = 1 << 20, 1000
    b = engine.synth(n=n, nflows=flows, len_a=1500, seed=0x5EED0001)
    tcb, live = rxg.synthetic_tcb_table(flows)
    engine.tcb_load(tcb, live)
    engine.tcb_sync()
    recs = engine.alloc(n * 16)
    engine.rx_burst_dev(b["arena"].ptr, b["off64"].ptr, b["len"].ptr, n, recs.ptr, rxg.REC16)
    cap = n * 1456
    arena, msgs, used = engine.alloc(cap), engine.alloc(n * 16), engine.alloc(8)
    engine.payload_gather_dev(arena.ptr, cap, msgs.ptr, used.ptr)
    engine.sync()
    assert int(used.download(np.uint64, 1)[0]) == cap
    m = msgs.download(rxg.PAYLOAD_MSG_DTYPE, n)
    assert (m["len"] == 1446).all() and (m["arena_off"] == np.arange(n, dtype=np.uint64) * 1456).all()
    assert (m["flags"] == (rxg.PM_GATHERED | rxg.PM_REF_OVERSIZE)).all()
    fr = b["arena"].download(np.uint8, n * 1536).reshape(n, 1536)
    ga = arena.download(np.uint8, cap).reshape(n, 1456)
    assert np.array_equal(ga[:, :1446], fr[:, 54:1500])
    assert not ga[:, 1446:].any()
    for d in (recs, arena, msgs, used):
        d.free()


def test_gather_c4_imix_full_size_property(engine):
    """BASELINE C4 batch (2^20 IMIX frames 64/576/1500, 64 K flows; payloads of 10, 522 and
    1 446 bytes mixed inside every workgroup): every payload gathered, messages packed in
    packet order at 16-byte-rounded offsets, each message's bytes equal to the frame's
    bytes 54..len and its padding zero."""
    n, flows = 1 << 20, 65536
    b = engine.synth(n=n, nflows=flows, mix=1, seed=0x5EED0004)
    tcb, live = rxg.synthetic_tcb_table(flows)
    engine.tcb_load(tcb, live)
    engine.tcb_sync()
    recs = engine.alloc(n * 16)
    engine.rx_burst_dev(b["arena"].ptr, b["off64"].ptr, b["len"].ptr, n, recs.ptr, rxg.REC16)
    lens = b["len"].download(np.uint16, n).astype(np.int64)
    off = b["off64"].download(np.uint32, n).astype(np.int64) * 64
    assert set(np.unique(lens)) == {64, 576, 1500}
    pl = lens - 54
    r16 = (pl + 15) // 16 * 16
    cap = int(r16.sum())
    arena, msgs, used = engine.alloc(cap), engine.alloc(n * 16), engine.alloc(8)
    engine.payload_gather_dev(arena.ptr, cap, msgs.ptr, used.ptr)
    engine.sync()
    assert int(used.download(np.uint64, 1)[0]) == cap
    m = msgs.download(rxg.PAYLOAD_MSG_DTYPE, n)
    exp_off = np.concatenate([[0], np.cumsum(r16)[:-1]]).astype(np.uint64)
    assert (m["len"] == pl).all() and (m["arena_off"] == exp_off).all()
    assert ((m["flags"] & rxg.PM_GATHERED) != 0).all()
    fr = b["arena"].download(np.uint8, b["arena_bytes"])
    ga = arena.download(np.uint8, cap)
    for L in (64, 576, 1500):  # one length class at a time, in chunks (host memory)
        idx = np.nonzero(lens == L)[0]
        P, R = L - 54, (L - 54 + 15) // 16 * 16
        for c in range(0, len(idx), 1 << 15):
            k = idx[c:c + (1 << 15)]
            src = fr[(off[k] + 54)[:, None] + np.arange(P)]
            dst = ga[exp_off[k].astype(np.int64)[:, None] + np.arange(R)]
            assert np.array_equal(dst[:, :P], src), f"payload bytes differ (length {L})"
            assert not dst[:, P:].any(), f"padding not zero (length {L})"
    for d in (recs, arena, msgs, used):
        d.free()


# ------------------------------------------------------------------ end to end ---
def multiflow_bursts(seed: int, nflows: int = 40, nseg: int = 10):
    """Clients connect, stream segments (some reordered, duplicated, or ending right at the
    window edge), FIN; frames of all flows interleaved in random bursts."""
    rng = random.Random(seed)
    syns, queues = [], []
    for k in range(nflows):
        src, sport = pktgen.ip4(10, 1, k >> 8, k & 255), 20000 + k
        isn = 0xFFFFFF00 + rng.randrange(200) if rng.random() < 0.1 else rng.getrandbits(32)
        isn = isn if isn != 0xFFFFFFFF else 7
        mk = lambda s, fl, p=b"": c1.raw_frame(src, c1.SERVER, sport, 80, s, 1, fl, p)  # noqa: E731
        syns.append(mk(isn, 0x02))
        seq = (isn + 1) & 0xFFFFFFFF
        segs = [mk(seq, 0x10)]
        data = []
        for _ in range(nseg):
            L = rng.choice([1, 7, 100, 512, 999, rng.randrange(1, 1000)])
            data.append((seq, rng.randbytes(L)))
            seq = (seq + L) & 0xFFFFFFFF
        frames = [mk(s, 0x18, p) for s, p in data]
        r = rng.random()
        if r < 0.2:                       # reordering
            i = rng.randrange(len(frames) - 1)
            frames[i], frames[i + 1] = frames[i + 1], frames[i]
        elif r < 0.35:                    # an old duplicate
            i = rng.randrange(1, len(frames))
            frames.insert(i + 1, frames[i - 1])
        elif r < 0.5:                     # retransmission of the latest (ends at cur)
            i = rng.randrange(len(frames))
            frames.insert(i + 1, frames[i])
        # (a bare FIN behind held pairs makes the reference's AdjustPair delete it and walk
        # off the list, tcp_windows.c:94-102: reordered flows end with a data-carrying FIN)
        fin_payload = rng.randbytes(rng.randrange(r < 0.2, 50)) if r < 0.2 or rng.random() < 0.5 else b""
        frames.append(mk(seq, 0x11, fin_payload))
        queues.append(segs + frames)
    rng.shuffle(syns)
    bursts = [syns]
    cur = []
    while any(queues):
        q = rng.choice([q for q in queues if q])
        cur.append(q.pop(0))
        if len(cur) >= rng.randrange(1, 200):
            bursts.append(cur)
            cur = []
    if cur:
        bursts.append(cur)
    return bursts


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_multiflow_exchange_equals_reference(engine, seed):
    bursts = multiflow_bursts(seed)
    ref = c1.drive_cpu(bursts)
    got = c1.drive_rxg(engine, bursts)
    assert got.rings == ref.rings                    # every socket-ring message, per TCB
    assert got.log == ref.log and got.rows == ref.rows
    assert {i: t["ack"] for i, t in got.tcb.items()} == {i: t["ack"] for i, t in ref.tcb.items()}
    assert got.sent == ref.sent
    # every segment an empty in-order window delivers whole came from the device gather
    assert got.taken == ref.eligible and got.eligible == 0 and got.taken > 200


def test_oversize_payloads_are_delivered_and_flagged(engine):
    """>= 1000-byte segments: the reference asserts in GetData (tcp_windows.c:170); rxg
    delivers them (RXG_PM_REF_OVERSIZE) — equal to the window restatement with the assert
    lifted."""
    msgs = [bytes([i]) * (1000 + 37 * i) for i in range(6)]
    bursts = c1.peer_script(msgs, False)
    with pytest.raises(ow.RefAbort):
        c1.drive_cpu(c1.peer_script(msgs, False))
    ref = c1.drive_cpu(bursts, oversize_ok=True)
    got = c1.drive_rxg(engine, c1.peer_script(msgs, False))
    assert got.ring == ref.ring == msgs and got.taken == len(msgs)
