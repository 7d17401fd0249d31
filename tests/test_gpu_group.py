"""GPU: several contexts behind one rx loop (include/rxg.h rxg_group_*).

The box has one GPU, so the groups here put two or three contexts on device 0: each member
still has its own stream, staging, mirror replica and counters, which is everything the
group logic touches (sharding, packet-order records, mirror broadcast, per-shard replay,
counter sum).  The expectations are the single-context burst and the sequential oracle of
tests/test_gpu_replay.py (the reference's ether_in loop, one packet at a time)."""
import ctypes as C
import random
import threading

import numpy as np
import pytest

import pktgen
import rxg
from test_gpu_replay import Model, scenario, sequential_reference

pytestmark = pytest.mark.gpu
MB = dict(max_batch=1 << 14, max_bytes=32 << 20)


def _ops(frames, bufs, got, model, add_mac=None):
    addr = {C.addressof(b): i for i, b in enumerate(bufs)}

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

    return rxg.HandoffOps(None, rxg.HANDOFF_FREE(free_mbuf), rxg.HANDOFF_ARP_IN(), rxg.HANDOFF_GET_MAC(),
                          rxg.HANDOFF_ADD_MAC(add_mac) if add_mac else rxg.HANDOFF_ADD_MAC(),
                          rxg.HANDOFF_SEND_RESET(rst), rxg.HANDOFF_ON_SEGMENT(),
                          rxg.HANDOFF_TCPSWITCH(tcpswitch))


@pytest.mark.parametrize("ndev", [2, 3])
def test_group_burst_equals_single_context(engine, ndev):
    rows, frames = scenario(5, n=1001)   # 1001: shards of 501/500 and 334/334/333
    tcb, live = pktgen.table_arrays(rows)
    engine.tcb_load(tcb, live)
    engine.counters_reset()
    single = engine.rx_burst(frames, rxg.REC48)
    scnt = engine.counters()
    with rxg.Group([0] * ndev, **MB) as g:
        assert len(g) == ndev
        g.tcb_load(tcb, live)
        g.counters_reset()
        for kind in (rxg.REC48, rxg.REC16, rxg.REC8):
            recs = g.rx_burst(frames, kind)
            want = {rxg.REC48: single, rxg.REC16: np.ascontiguousarray(single["c"]),
                    rxg.REC8: rxg.rec8_pack(single["c"])}[kind]
            assert recs.tobytes() == want.tobytes()
        assert g.counters().tolist() == (3 * scnt).tolist()
        # fewer frames than members: empty shards are bursts of nothing
        one = g.rx_burst(frames[:1], rxg.REC48)
        assert one.tobytes() == single[:1].tobytes()
        assert len(g.rx_burst([], rxg.REC48)) == 0


@pytest.mark.parametrize("ndev,seed,kind", [(2, 1, rxg.REC16), (3, 2, rxg.REC16), (2, 3, rxg.REC16),
                                            (3, 4, rxg.REC8)])
def test_group_replay_sequential_equivalence(ndev, seed, kind):
    """Handlers write through the group, so a write made while replaying shard i reaches the
    members of shards i+1.. before their replay, which re-classifies what it affects."""
    rows, frames = scenario(seed)
    exp, ecnt, erows = sequential_reference(rows, frames)
    tcb, live = pktgen.table_arrays(rows)
    with rxg.Group([0] * ndev, **MB) as g:
        g.tcb_load(tcb, live)
        g.counters_reset()
        recs = g.rx_burst(frames, kind)
        model = Model(rows, g)
        bufs = [C.create_string_buffer(f, max(len(f), 64)) for f in frames]
        got = [None] * len(frames)
        ops = _ops(frames, bufs, got, model)
        ptrs = (C.c_void_p * len(bufs))(*[C.addressof(b) for b in bufs])
        g.rx_replay(ops, ptrs, ptrs, recs.ctypes.data, len(bufs), kind)
        for i, (v, idx, st) in enumerate(exp):
            if v == rxg.V_DISPATCH:
                assert got[i] == ("switch", idx, st), (i, got[i], exp[i])
            elif v in (rxg.V_RST_NOPCB, rxg.V_RST_LISTEN_NONSYN):
                assert got[i] == ("rst",), (i, got[i], exp[i])
        assert model.rows == erows
        assert g.counters().tolist() == ecnt.tolist()
        # every member's mirror ends as the reference's table: a burst of the same frames on
        # each member equals the oracle against the final rows
        t2, l2 = pktgen.table_arrays(erows)
        with rxg.Engine(0, **MB) as ref:
            ref.tcb_load(t2, l2)
            want = ref.rx_burst(frames, rxg.REC16)
        for m in g.members:
            assert m.rx_burst(frames, rxg.REC16).tobytes() == want.tobytes()
        assert g.replaying() == -1


def test_group_arp_learn_once_across_shards():
    """ip.c:30-32 with the ARP mirror on a group: a source first seen in shard 0 is learned
    there; the group tells every member, so shard 1 does not learn it again, even though the
    caller's add_mac makes no mirror call of its own."""
    rng = random.Random(4)
    known = [pktgen.ip4(10, 0, 0, k) for k in range(8)]
    unknown = [pktgen.ip4(10, 9, 0, k) for k in range(24)]
    frames = [pktgen.frame(src_ip=rng.choice(known if rng.random() < 0.4 else unknown),
                           sport=rng.randrange(65536), flags=0x10) for _ in range(600)]
    tcb, live = pktgen.table_arrays([(80, 0, pktgen.raw_of_host(pktgen.ip4(192, 168, 78, 2)), 0, 1)])
    exp, seen = [], set(known)
    for f in frames:
        src = int.from_bytes(f[26:30], "big")
        if src not in seen:
            seen.add(src)
            exp.append(src)
    calls = []

    def add_mac(u, ip, mac):
        calls.append(ip)
        return 1

    with rxg.Group([0, 0, 0], **MB) as g:
        g.tcb_load(tcb, live)
        g.arp_load(known)
        recs = g.rx_burst(frames, rxg.REC16)
        bufs = [C.create_string_buffer(f, max(len(f), 64)) for f in frames]
        got = [None] * len(frames)
        ops = _ops(frames, bufs, got, Model([]), add_mac=add_mac)
        ptrs = (C.c_void_p * len(bufs))(*[C.addressof(b) for b in bufs])
        g.rx_replay(ops, ptrs, ptrs, recs.ctypes.data, len(bufs), 16)
        assert calls == exp
        assert all(m.arp_count() == len(known) + len(exp) for m in g.members)


def test_group_posted_writes_and_errors():
    dst = pktgen.raw_of_host(pktgen.ip4(192, 168, 78, 2))
    f = pktgen.frame(src_ip=pktgen.ip4(10, 1, 0, 1), dst_ip=pktgen.ip4(192, 168, 78, 2), sport=1234,
                     dport=80, flags=0x10)
    with rxg.Group([0, 0], **MB) as g:
        # app threads post; the next group burst applies the writes on every member
        ths = [threading.Thread(target=lambda k=k: g.tcb_post_upsert(k, 9000 + k, 1, dst, 7, 4))
               for k in range(4)]
        [t.start() for t in ths]
        [t.join() for t in ths]
        assert g.tcb_post_upsert(4, 80, 1234, dst, pktgen.ip4(10, 1, 0, 1), 4) == 0
        recs = g.rx_burst([f, f, f], rxg.REC16)
        assert (recs["tcb_idx"] == 4).all() and (recs["verdict"] == rxg.V_DISPATCH).all()
        assert all(m.tcb_count() == 5 for m in g.members)
        # a replay must follow a group burst of the same n
        ops = rxg.HandoffOps()
        bufs = (C.c_void_p * 2)()
        with pytest.raises(rxg.RxgError, match="last group burst"):
            g.rx_replay(ops, bufs, bufs, recs.ctypes.data, 2, 16)
        # a member error carries the member's text
        with pytest.raises(rxg.RxgError, match="member 0: .*index"):
            g.tcb_set_state(-3, 1)
        # shards above max_batch fail the burst, and a replay of it is refused
        big = [f] * (2 * (1 << 14) + 2)
        with pytest.raises(rxg.RxgError, match="max_batch"):
            g.rx_burst(big, rxg.REC16)
        recs = np.zeros(len(big), dtype=rxg.REC16_DTYPE)
        ptrs = (C.c_void_p * len(big))()
        with pytest.raises(rxg.RxgError, match="last group burst failed"):
            g.rx_replay(ops, ptrs, ptrs, recs.ctypes.data, len(big), 16)


def test_group_counter_merge_rccl():
    """rxg_group_counters_read merges with an RCCL all-reduce when the members are distinct
    GPUs (one rank each; every GPU of the box, one on the test box) and on the host when
    they share one; both equal the oracle's counters of the burst, and a second merge does
    not double-count (the all-reduce writes a separate block)."""
    import oracle
    import torch
    rows, frames = scenario(9, n=1500, closed=0.05)
    tcb, live = pktgen.table_arrays(rows)
    arena, off, lens = pktgen.pack_arena(frames)
    _, ecnt = oracle.rx_batch(arena, off, lens, tcb, live)
    for devs, rccl in ((list(range(torch.cuda.device_count())), True), ([0, 0], False)):
        with rxg.Group(devs, **MB) as g:
            assert g.counters_rccl() == rccl
            assert (g.counters_rccl_why() == "") == rccl, g.counters_rccl_why()
            g.tcb_load(tcb, live)
            g.counters_reset()
            g.rx_burst(frames, rxg.REC16)
            assert g.counters().tolist() == ecnt.tolist()
            assert g.counters().tolist() == ecnt.tolist()
            g.rx_burst(frames, rxg.REC16)
            assert g.counters().tolist() == (2 * ecnt).tolist()


def _dev_shards(g, frames, cuts, kind):
    """Member i's share frames[cuts[i]:cuts[i+1]] packed into member i's device memory."""
    shards, keep = [], []
    for i, m in enumerate(g.members):
        part = frames[cuts[i]:cuts[i + 1]]
        arena, off, lens = pktgen.pack_arena(part) if part else pktgen.pack_arena([pktgen.frame()])
        da, do, dl = m.to_device(arena), m.to_device(off), m.to_device(lens)
        dout = m.alloc(max(len(part), 1) * kind)
        keep.append((m, da, do, dl, dout, len(part)))
        shards.append((da.ptr, do.ptr, dl.ptr, len(part), dout.ptr))
    return shards, keep


@pytest.mark.parametrize("ndev,seed,kind", [(2, 11, rxg.REC16), (3, 12, rxg.REC8), (3, 13, rxg.REC16)])
def test_group_dev_burst_replay_sequential_equivalence(ndev, seed, kind):
    """rxg_group_rx_burst_dev: each member's contiguous share already in its GPU's memory
    (uneven shares, one empty), every member launched at once; the records equal the host
    group burst's, and burst + replay in global packet order equals the reference's
    sequential ether_in loop under in-burst SYN / FIN / remove writes (main.c:391-399)."""
    rng = random.Random(seed)
    rows, frames = scenario(seed)
    exp, ecnt, erows = sequential_reference(rows, frames)
    tcb, live = pktgen.table_arrays(rows)
    n = len(frames)
    cuts = [0] + sorted(rng.sample(range(1, n), ndev - 1)) + [n]
    if ndev == 3:
        cuts[2] = cuts[1]  # member 1 gets nothing
    with rxg.Group([0] * ndev, **MB) as g:
        g.tcb_load(tcb, live)
        want = g.rx_burst(frames, kind)  # the host-buffer group burst, same table
        g.counters_reset()
        shards, keep = _dev_shards(g, frames, cuts, kind)
        try:
            g.rx_burst_dev(shards, kind)
            g.sync()
            recs = np.concatenate([dout.download(rxg.rec_dtype(kind), k) for (_, _, _, _, dout, k) in keep])
            assert recs.tobytes() == want.tobytes()
            model = Model(rows, g)
            bufs = [C.create_string_buffer(f, max(len(f), 64)) for f in frames]
            got = [None] * n
            ops = _ops(frames, bufs, got, model)
            ptrs = (C.c_void_p * n)(*[C.addressof(b) for b in bufs])
            g.rx_replay(ops, ptrs, ptrs, recs.ctypes.data, n, kind)
        finally:
            for (m, *bufs_) in keep:
                for d in bufs_[:4]:
                    d.free()
    for i, (v, idx, st) in enumerate(exp):
        if v == rxg.V_DISPATCH:
            assert got[i] == ("switch", idx, st), (i, got[i], exp[i])
        elif v in (rxg.V_RST_NOPCB, rxg.V_RST_LISTEN_NONSYN):
            assert got[i] == ("rst",), (i, got[i], exp[i])
    assert model.rows == erows


def test_group_dev_burst_arguments():
    with rxg.Group([0, 0], **MB) as g:
        with pytest.raises(rxg.RxgError, match="1 shards for 2 members"):
            g.rx_burst_dev([(0, 0, 0, 0, 0)], rxg.REC16)
        arr = (rxg.DevBatch * 2)(rxg.DevBatch(0, 0, 0, 0, rxg.REC16, 0), rxg.DevBatch(0, 0, 0, 0, rxg.REC8, 0))
        assert rxg.load_library().rxg_group_rx_burst_dev(g.g, arr, 2) == -22
        assert b"rec_kind" in rxg.load_library().rxg_group_last_error()
        # a failed group burst leaves nothing to replay
        ops = rxg.HandoffOps()
        ptrs = (C.c_void_p * 1)()
        recs = np.zeros(1, dtype=rxg.REC16_DTYPE)
        with pytest.raises(rxg.RxgError, match="last group burst failed"):
            g.rx_replay(ops, ptrs, ptrs, recs.ctypes.data, 0, 16)
