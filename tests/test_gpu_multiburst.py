"""GPU: several bursts of one frame pool in one launch (rxg_rx_bursts_dev).

* Records and counters equal k single-burst launches and the oracle, for bursts of mixed
  sizes (1 frame, a partial last slice, an empty burst, all-small slices next to class
  slices) whose frames are interleaved in the pool, and for more bursts than one launch
  takes (kMaxBursts = 32).
* The launch's bursts replayed in order (one rxg_rx_replay each) equal the reference's
  sequential ether_in loop over their concatenation while the handlers write tcbs[]: a
  burst sees the writes its predecessors' replays made (tcp_listen children, remove_tcb,
  state changes; tcp_states.c:150-219).
* A payload gather between replays covers the burst to be replayed next.
* The same with 8-byte records (RXG_REC8): the kernel's packing equals the oracle's record
  packed (rxg.rec8_pack), and replay and gather read them.
"""
import ctypes as C
import random

import numpy as np
import pytest

import oracle
import pktgen
import rxg
from test_gpu_replay import Model, scenario, sequential_reference

pytestmark = pytest.mark.gpu


def _pool(frames, order):
    """Frames packed into one pool in `order` (a permutation), so bursts interleave."""
    slots = [(len(f) + 63) // 64 for f in frames]
    off = np.zeros(len(frames), dtype=np.uint32)
    pos = 0
    for i in order:
        off[i] = pos
        pos += slots[i]
    arena = np.full(max(pos, 1) * 64, 0xA5, dtype=np.uint8)
    for i, f in enumerate(frames):
        o = int(off[i]) * 64
        arena[o:o + len(f)] = np.frombuffer(f, dtype=np.uint8)
    return arena, off


def _cuts(rng, n, k):
    c = sorted(rng.sample(range(1, n), k - 1))
    return [0] + c + [n]


@pytest.mark.parametrize("k,seed,kind", [(5, 1, rxg.REC48), (40, 2, rxg.REC48), (5, 3, rxg.REC8), (40, 4, rxg.REC8)])
def test_multi_burst_records_equal_single_bursts_and_oracle(engine, k, seed, kind):
    rng = random.Random(seed)
    rows, frames = pktgen.parity_set(seed=100 + seed, n=6000)
    # a run of small frames so all-small slices appear inside some bursts
    frames[1000:1400] = [pktgen.frame(sport=2000 + i % 7, payload=bytes(i % 10)) for i in range(400)]
    tcb, live = pktgen.table_arrays(rows)
    engine.tcb_load(tcb, live)
    n = len(frames)
    cuts = _cuts(rng, n, k)
    cuts[2] = cuts[1]                      # an empty burst
    if k > 3:
        cuts[3] = cuts[2] + 1              # a one-frame burst
    order = list(range(n))
    rng.shuffle(order)
    arena, off = _pool(frames, order)
    lens = np.array([len(f) for f in frames], dtype=np.uint16)
    d_arena = engine.to_device(arena)
    dev = []
    try:
        bursts = []
        for j in range(k):
            a, b = cuts[j], cuts[j + 1]
            do = engine.to_device(off[a:b] if b > a else np.zeros(1, np.uint32))
            dl = engine.to_device(lens[a:b] if b > a else np.zeros(1, np.uint16))
            dout = engine.alloc(max(b - a, 1) * kind)
            dev += [do, dl, dout]
            bursts.append((do.ptr, dl.ptr, b - a, dout.ptr))
        engine.counters_reset()
        engine.rx_bursts_dev(d_arena.ptr, bursts, kind)
        engine.sync()
        cnt = engine.counters()
        got = np.concatenate([dev[3 * j + 2].download(rxg.rec_dtype(kind), cuts[j + 1] - cuts[j]) for j in range(k)])
        parr, poff, plens = pktgen.pack_arena(frames)
        exp, ecnt = oracle.rx_batch(parr, poff, plens, tcb, live)
        if kind == rxg.REC8:
            exp = rxg.rec8_pack(exp["c"])
        assert got.tobytes() == exp.tobytes()
        assert cnt.tolist() == ecnt.tolist()
        # one burst at a time through the single-burst entry point: the same records
        single = np.concatenate([engine.rx_arena(*pktgen.pack_arena(frames[cuts[j]:cuts[j + 1]]), kind)
                                 for j in range(k)])
        assert single.tobytes() == got.tobytes()
    finally:
        for d in dev + [d_arena]:
            d.free()


@pytest.mark.parametrize("seed,kind", [(4, rxg.REC16), (5, rxg.REC16), (6, rxg.REC8)])
def test_multi_burst_replay_sequential_equivalence(replay_engine, seed, kind):
    engine = replay_engine
    rows, frames = scenario(seed, n=1500, closed=0.05)
    exp, ecnt, erows = sequential_reference(rows, frames)
    tcb, live = pktgen.table_arrays(rows)
    engine.tcb_load(tcb, live)
    engine.tcb_sync()
    rng = random.Random(seed)
    k = 7
    cuts = _cuts(rng, len(frames), k)
    order = list(range(len(frames)))
    rng.shuffle(order)
    arena, off = _pool(frames, order)
    lens = np.array([len(f) for f in frames], dtype=np.uint16)
    d_arena = engine.to_device(arena)
    dev, bursts = [], []
    for j in range(k):
        a, b = cuts[j], cuts[j + 1]
        do, dl, dout = engine.to_device(off[a:b]), engine.to_device(lens[a:b]), engine.alloc((b - a) * kind)
        dev += [do, dl, dout]
        bursts.append((do.ptr, dl.ptr, b - a, dout.ptr))
    model = Model(rows, engine)
    bufs = [C.create_string_buffer(f, max(len(f), 64)) for f in frames]
    addr = {C.addressof(b): i for i, b in enumerate(bufs)}
    got = [None] * len(frames)

    def free_mbuf(u, m):
        i = addr[m]
        if got[i] is None:
            got[i] = ("free",)

    def rst(u, ip, tcp):
        got[addr[ip - 14]] = ("rst",)

    def tcpswitch(u, idx, st, tcp, ip, m):
        i = addr[m]
        got[i] = ("switch", idx, st)
        model.handle(idx, st, frames[i])
        return 0

    ops = rxg.HandoffOps(None, rxg.HANDOFF_FREE(free_mbuf), rxg.HANDOFF_ARP_IN(), rxg.HANDOFF_GET_MAC(),
                         rxg.HANDOFF_ADD_MAC(), rxg.HANDOFF_SEND_RESET(rst), rxg.HANDOFF_ON_SEGMENT(),
                         rxg.HANDOFF_TCPSWITCH(tcpswitch))
    lib = rxg.load_library()
    try:
        engine.counters_reset()
        engine.rx_bursts_dev(d_arena.ptr, bursts, kind)
        engine.sync()
        for j in range(k):
            a, b = cuts[j], cuts[j + 1]
            recs = dev[3 * j + 2].download(rxg.rec_dtype(kind), b - a)
            ptrs = (C.c_void_p * (b - a))(*[C.addressof(x) for x in bufs[a:b]])
            rc = lib.rxg_rx_replay(engine.ctx, C.byref(ops), ptrs, ptrs, recs.ctypes.data, b - a, kind)
            assert rc == 0, lib.rxg_last_error()
        for i, (v, idx, st) in enumerate(exp):
            if v == rxg.V_DISPATCH:
                assert got[i] == ("switch", idx, st), (i, got[i], exp[i])
            elif v in (rxg.V_RST_NOPCB, rxg.V_RST_LISTEN_NONSYN):
                assert got[i] == ("rst",), (i, got[i], exp[i])
            else:
                assert got[i] == ("free",), (i, got[i], exp[i])
        assert model.rows == erows
        assert engine.counters().tolist() == ecnt.tolist()
        # replaying out of order is refused (the next burst has another size)
        if cuts[2] - cuts[1] != cuts[1] - cuts[0]:
            recs0 = dev[2].download(rxg.rec_dtype(kind), cuts[1])
            ptrs = (C.c_void_p * cuts[1])(*[C.addressof(x) for x in bufs[:cuts[1]]])
            engine.rx_bursts_dev(d_arena.ptr, bursts, kind)
            engine.sync()
            none = rxg.HandoffOps()  # no handlers: only the cursor is under test here
            assert lib.rxg_rx_replay(engine.ctx, C.byref(none), ptrs, ptrs, recs0.ctypes.data, cuts[1], kind) == 0
            assert lib.rxg_rx_replay(engine.ctx, C.byref(none), ptrs, ptrs, recs0.ctypes.data, cuts[1], kind) == -22
    finally:
        for d in dev + [d_arena]:
            d.free()


@pytest.mark.parametrize("kind", [rxg.REC16, rxg.REC8])
def test_multi_burst_gather_follows_the_replay_cursor(engine, kind):
    """rxg_payload_gather_dev after a multi-burst launch gathers the burst to be replayed
    next; after that burst's replay, the next one."""
    rng = random.Random(8)
    frames = [pktgen.frame(sport=3000 + i, payload=rng.randbytes(rng.randrange(0, 300))) for i in range(900)]
    tcb, live = pktgen.table_arrays([(80, 0, pktgen.raw_of_host(pktgen.ip4(192, 168, 78, 2)), 0, 1)])
    engine.tcb_load(tcb, live)
    cuts = [0, 300, 700, 900]
    arena, off = _pool(frames, list(range(len(frames))))
    lens = np.array([len(f) for f in frames], dtype=np.uint16)
    d_arena = engine.to_device(arena)
    dev, bursts = [], []
    for j in range(3):
        a, b = cuts[j], cuts[j + 1]
        do, dl, dout = engine.to_device(off[a:b]), engine.to_device(lens[a:b]), engine.alloc((b - a) * kind)
        dev += [do, dl, dout]
        bursts.append((do.ptr, dl.ptr, b - a, dout.ptr))
    from oracle import payload as opl
    lib = rxg.load_library()
    ops = rxg.HandoffOps()
    bufs = [C.create_string_buffer(f, max(len(f), 64)) for f in frames]
    try:
        engine.rx_bursts_dev(d_arena.ptr, bursts, kind)
        engine.sync()
        for j in range(3):
            a, b = cuts[j], cuts[j + 1]
            recs = dev[3 * j + 2].download(rxg.rec_dtype(kind), b - a)
            r16 = rxg.rec8_expand(recs) if kind == rxg.REC8 else recs
            e_msgs, e_arena, e_used = opl.gather(frames[a:b], r16, 1 << 40)
            g_arena, g_msgs, g_used = engine.payload_gather(b - a, e_used)
            assert g_used == e_used and g_msgs.tobytes() == e_msgs.tobytes()
            assert g_arena[:len(e_arena)].tobytes() == e_arena.tobytes()
            ptrs = (C.c_void_p * (b - a))(*[C.addressof(x) for x in bufs[a:b]])
            assert lib.rxg_rx_replay(engine.ctx, C.byref(ops), ptrs, ptrs, recs.ctypes.data, b - a, kind) == 0
    finally:
        for d in dev + [d_arena]:
            d.free()


@pytest.mark.parametrize("kind", [rxg.REC8, rxg.REC48])
def test_carried_patches_reach_every_launch_of_a_multi_burst_call(kind):
    """tcbs[] writes made just before a call of more bursts than one launch takes (40 >
    kMaxBursts = 32): the call's first launch carries the patch list and the
    second, queued behind it on the context's stream, must classify against the patched table
    too.  Every burst's records and the counters equal the oracle over the table after the
    writes (remove_tcb tcp_tcb.c:175-186, state changes, a re-tupled slot)."""
    # a fresh context: no table reader pending on another stream, so the list is carried
    engine = rxg.Engine(device=0)
    rng = random.Random(808)
    rows, frames = pktgen.parity_set(seed=808, n=6000)
    tcb, live = pktgen.table_arrays(rows)
    engine.tcb_load(tcb, live)
    engine.tcb_sync()
    engine.sync()
    live = live.copy()
    tcb = tcb.copy()
    for i in rng.sample([x for x in range(1, len(tcb)) if live[x]], 12):  # a short list: carried
        if rng.random() < 0.5:
            live[i] = 0
            engine.tcb_remove(i)
        else:
            st = rng.choice([rxg.LISTENING, rxg.TCP_ESTABLISHED, rxg.SYN_RECV])
            tcb["state"][i] = st
            engine.tcb_set_state(i, st)
    n, k = len(frames), 40
    cuts = _cuts(rng, n, k)
    order = list(range(n))
    rng.shuffle(order)
    arena, off = _pool(frames, order)
    lens = np.array([len(f) for f in frames], dtype=np.uint16)
    d_arena = engine.to_device(arena)
    dev, bursts = [], []
    try:
        for j in range(k):
            a, b = cuts[j], cuts[j + 1]
            do, dl, dout = engine.to_device(off[a:b]), engine.to_device(lens[a:b]), engine.alloc((b - a) * kind)
            dev += [do, dl, dout]
            bursts.append((do.ptr, dl.ptr, b - a, dout.ptr))
        engine.counters_reset()
        engine.sync()
        engine.rx_bursts_dev(d_arena.ptr, bursts, kind)
        engine.sync()
        got = np.concatenate([dev[3 * j + 2].download(rxg.rec_dtype(kind), cuts[j + 1] - cuts[j]) for j in range(k)])
        parr, poff, plens = pktgen.pack_arena(frames)
        exp, ecnt = oracle.rx_batch(parr, poff, plens, tcb, live)
        if kind == rxg.REC8:
            exp = rxg.rec8_pack(exp["c"])
        assert got.tobytes() == exp.tobytes()
        assert engine.counters().tolist() == ecnt.tolist()
    finally:
        for d in dev + [d_arena]:
            d.free()
        engine.close()
