"""GPU: randomized multi-burst runs against the sequential reference loop.

A stream of frames (SYN/ACK/FIN traffic from the replay scenario) is cut into bursts of
random sizes (1..400).  Between bursts an "application thread" posts random tcbs[] writes
(rxg_tcb_post: new listeners, state changes, removals, re-tuples of live slots) that the
reference would have made before the burst's first packet; inside bursts the handlers
make tcp_states.c-shaped writes (tests/test_gpu_replay.py Model).  Every packet's outcome
and the final table must equal the oracle run one packet at a time with the same writes
at the same points."""
import ctypes as C
import os
import random

import pytest

import oracle
import pktgen
import rxg
from test_gpu_replay import LISTENING, Model, scenario

pytestmark = pytest.mark.gpu


def _random_ops(rng, rows, dst_raw):
    """A few posted writes, each valid given the ones before it: (kind, idx, value)."""
    ops, live, nxt = [], [i for i, r in enumerate(rows) if r is not None], len(rows)
    cur = {i: rows[i] for i in live}
    for _ in range(rng.randrange(0, 6)):
        k = rng.random()
        if k < 0.25:    # a new listener appended (alloc_tcb + socket_bind + listen)
            v = (rng.choice([80, 8080, 9000]), 0, dst_raw, 0, LISTENING)
            ops.append(("up", nxt, v))
            live.append(nxt)
            cur[nxt] = v
            nxt += 1
        elif k < 0.5 and live:   # state change
            i = rng.choice(live)
            st = rng.choice([0, 1, 3, 4])
            ops.append(("st", i, st))
            cur[i] = cur[i][:4] + (st,)
        elif k < 0.7 and len(live) > 1:   # removal (slot 0 stays: one listener)
            i = rng.choice(live[1:])
            ops.append(("rm", i, None))
            live.remove(i)
            del cur[i]
        elif live:               # re-tuple a live slot (socket_connect-style rewrite)
            i = rng.choice(live)
            r = cur[i]
            v = (r[0], rng.choice([r[1], 40000 + rng.randrange(60)]), r[2], r[3], r[4])
            ops.append(("up", i, v))
            cur[i] = v
    return ops


def _apply(rows, ops):
    for kind, i, v in ops:
        if kind == "up":
            while len(rows) <= i:
                rows.append(None)
            rows[i] = v
        elif kind == "st":
            if rows[i] is not None:
                rows[i] = rows[i][:4] + (v,)
        elif kind == "rm":
            rows[i] = None


def _post(engine, ops):
    for kind, i, v in ops:
        if kind == "up":
            assert engine.tcb_post_upsert(i, v[0], v[1], v[2] & 0xFFFFFFFF, v[3] & 0xFFFFFFFF, v[4]) == 0
        elif kind == "st":
            assert engine.tcb_post_set_state(i, v) == 0
        else:
            assert engine.tcb_post_remove(i) == 0


# RXG_FUZZ_SEEDS=<k> adds k more seeds (soak runs; the regular suite runs these three)
_EXTRA = [(1000 + i, i % 3 == 0) for i in range(int(os.environ.get("RXG_FUZZ_SEEDS", "0")))]


@pytest.mark.parametrize("seed,arp", [(101, False), (202, False), (303, True)] + _EXTRA)
def test_random_bursts_equal_sequential_reference(replay_engine, seed, arp):
    engine = replay_engine
    """arp: the ARP mirror is on (half the sources known up front); the replay's add_mac
    calls must be the reference's ip_in learns (ip.c:30-32), first sighting in stream
    order, across bursts."""
    rng = random.Random(seed)
    rows, frames = scenario(seed, n=2500)
    dst_raw = rows[0][2]
    # cut into bursts and draw each burst's posted writes
    cuts, i = [], 0
    while i < len(frames):
        k = rng.choice([1, 2, 7, 32, 64, 150, 400])
        cuts.append((i, min(len(frames), i + k)))
        i += k
    # reference: one packet at a time, the posted writes applied before each burst
    ref_rows = list(rows)
    model = Model(ref_rows)
    plan, exp = [], []
    for b0, b1 in cuts:
        ops = _random_ops(rng, model.rows, dst_raw)
        plan.append(ops)
        _apply(model.rows, ops)
        for f in frames[b0:b1]:
            arena, off, lens = pktgen.pack_arena([f])
            tcb, live = pktgen.table_arrays(model.rows)
            rec, _ = oracle.rx_batch(arena, off, lens, tcb, live)
            r = rec[0]["c"]
            exp.append((int(r["verdict"]), int(r["tcb_idx"]), int(r["state"])))
            if r["verdict"] == rxg.V_DISPATCH:
                model.handle(int(r["tcb_idx"]), int(r["state"]), f)
    # ip_in's learns: every TCP packet (all of the scenario's frames) from an unknown source
    srcs = [int.from_bytes(f[26:30], "big") for f in frames]
    known = sorted(set(srcs))[::2] if arp else []
    exp_learn, seen = [], set(known)
    for sip in srcs:
        if sip not in seen:
            seen.add(sip)
            exp_learn.append(sip)
    # rxg: posts between bursts, handlers mirror inside them
    tcb, live = pktgen.table_arrays(rows)
    engine.tcb_load(tcb, live)
    engine.tcb_sync()
    learned = []
    if arp:
        engine.arp_load(known)
    else:
        engine.arp_disable()
    gm = Model(list(rows), engine)
    bufs = [C.create_string_buffer(f, max(len(f), 64)) for f in frames]
    addr = {C.addressof(b): i for i, b in enumerate(bufs)}
    got = [None] * len(frames)

    def free_mbuf(u, m):
        if got[addr[m]] is None:
            got[addr[m]] = ("free",)

    def rst(u, ip, tcp):
        got[addr[ip - 14]] = ("rst",)

    def tcpswitch(u, idx, st, tcp, ip, m):
        i = addr[m]
        got[i] = ("switch", idx, st)
        gm.handle(idx, st, frames[i])
        return 0

    def add_mac(u, ip, mac):
        learned.append(ip)
        return 1

    ops_t = rxg.HandoffOps(None, rxg.HANDOFF_FREE(free_mbuf), rxg.HANDOFF_ARP_IN(), rxg.HANDOFF_GET_MAC(),
                           rxg.HANDOFF_ADD_MAC(add_mac) if arp else rxg.HANDOFF_ADD_MAC(),
                           rxg.HANDOFF_SEND_RESET(rst), rxg.HANDOFF_ON_SEGMENT(),
                           rxg.HANDOFF_TCPSWITCH(tcpswitch))
    lib = rxg.load_library()
    for (b0, b1), ops in zip(cuts, plan):
        _post(engine, ops)
        _apply(gm.rows, ops)
        recs = engine.rx_burst(frames[b0:b1], rxg.REC16)
        ptrs = (C.c_void_p * (b1 - b0))(*[C.addressof(b) for b in bufs[b0:b1]])
        rc = lib.rxg_rx_replay(engine.ctx, C.byref(ops_t), ptrs, ptrs, recs.ctypes.data, b1 - b0, 16)
        assert rc == 0, lib.rxg_last_error()
    for i, (v, idx, st) in enumerate(exp):
        if v == rxg.V_DISPATCH:
            assert got[i] == ("switch", idx, st), (i, got[i], exp[i])
        elif v in (rxg.V_RST_NOPCB, rxg.V_RST_LISTEN_NONSYN):
            assert got[i] == ("rst",), (i, got[i], exp[i])
        else:
            assert got[i] == ("free",), (i, got[i], exp[i])
    assert gm.rows == model.rows
    if arp:
        assert learned == exp_learn
        assert engine.arp_count() == len(known) + len(exp_learn)
        engine.arp_disable()
    # the device mirror ends as the reference's table
    t2, l2 = pktgen.table_arrays(model.rows)
    want, _ = oracle.rx_batch(*pktgen.pack_arena(frames[:500]), t2, l2)
    assert engine.rx_burst(frames[:500], rxg.REC48).tobytes() == want.tobytes()
