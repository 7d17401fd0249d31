"""Flow-affinity sharding on the GPU (rxg_flow_partition): n contexts, each the
rx queue of one RSS partition with 1/n of the exact-tuple table, classify the frames steered
to them exactly as one context over the whole table does (the oracle, tcp_tcb.c:127-173):
listeners, the NULL slot in front of a listener, duplicate tuples, host-order dst, bad int
ports -- before and after mirror writes applied to every context."""
import random

import numpy as np
import pytest

import oracle
import pktgen
import rxg

pytestmark = pytest.mark.gpu


def _run_parts(engines, frames, tcb, live, rec_kind):
    n = len(engines)
    parts = [rxg.flow_part_of(f, n) for f in frames]
    for p, eng in enumerate(engines):
        idx = [i for i, q in enumerate(parts) if q == p]
        sub = [frames[i] for i in idx]
        arena, off, lens = pktgen.pack_arena(sub)
        eng.counters_reset()
        got = eng.rx_arena(arena, off, lens, rec_kind)
        exp, ecnt = oracle.rx_batch(arena, off, lens, tcb, live)
        exp = rxg.rec8_pack(exp["c"]) if rec_kind == rxg.REC8 else exp["c"]
        assert got.tobytes() == exp.tobytes(), f"partition {p} of {n}: records differ"
        assert np.array_equal(eng.counters(), ecnt), f"partition {p} of {n}: counters differ"
    return parts


@pytest.mark.parametrize("nparts", [2, 3])
@pytest.mark.parametrize("rec_kind", [rxg.REC8, rxg.REC16])
def test_flow_partitions_equal_whole_table(nparts, rec_kind):
    rows, frames = pktgen.parity_set(seed=60 + nparts, n=6000, nflows=2000)
    tcb, live = pktgen.table_arrays(rows)
    engines = [rxg.Engine(device=0) for _ in range(nparts)]
    whole = rxg.Engine(device=0)
    try:
        whole.tcb_load(tcb, live)
        whole.tcb_sync()
        for p, eng in enumerate(engines):
            eng.flow_partition(p, nparts)
            eng.tcb_load(tcb, live)
            eng.tcb_sync()
        keys = [eng.tcb_keys() for eng in engines]
        assert sum(keys) == whole.tcb_keys()               # every tuple in exactly one table
        assert min(keys) > 0.7 * whole.tcb_keys() / nparts  # and spread over them
        parts = _run_parts(engines, frames, tcb, live, rec_kind)
        assert len(set(parts)) == nparts

        # mirror writes, applied to every context: a new child on the listener's port, a
        # removed flow, a state change, the NULL slot in front of :8080 filled (the pass-2
        # NULL flag moves), a re-tupled slot
        rng = random.Random(nparts)
        tl = [list(r) if r is not None else None for r in rows]
        writes = []
        for k in range(40):
            i = rng.randrange(1, len(tl))
            if tl[i] is None:
                continue
            if k % 3 == 0:
                writes.append(("remove", i))
                tl[i] = None
            elif k % 3 == 1:
                writes.append(("state", i, pktgen.LISTENING if k % 2 else pktgen.ESTABLISHED))
                tl[i][4] = writes[-1][2]
            else:
                t = (80, 30000 + k, tl[i][2], pktgen.ip4(10, 200, k, 1), pktgen.ESTABLISHED)
                writes.append(("upsert", i, t))
                tl[i] = list(t)
        nul = next(i for i, r in enumerate(tl) if r is None)
        t = (9090, 1, pktgen.raw_of_host(pktgen.ip4(192, 168, 78, 2)), pktgen.ip4(10, 1, 2, 3), pktgen.ESTABLISHED)
        writes.append(("upsert", nul, t))
        tl[nul] = list(t)
        for eng in engines:
            for w in writes:
                if w[0] == "remove":
                    eng.tcb_remove(w[1])
                elif w[0] == "state":
                    eng.tcb_set_state(w[1], w[2])
                else:
                    d, s, dst, src, st = w[2]
                    eng.tcb_upsert(w[1], d, s, dst, src, st, identifier=(w[1] % 65535) + 1)
            eng.tcb_sync()
        rows2 = [tuple(r) if r is not None else None for r in tl]
        tcb2, live2 = pktgen.table_arrays(rows2)
        _run_parts(engines, frames, tcb2, live2, rec_kind)
    finally:
        for eng in engines:
            eng.close()
        whole.close()


def test_group_refuses_partitioned_members():
    rows, frames = pktgen.parity_set(seed=70, n=200)
    tcb, live = pktgen.table_arrays(rows)
    with rxg.Group([0, 0], max_batch=4096, max_bytes=8 << 20) as g:
        g.tcb_load(tcb, live)
        g.rx_burst(frames, rxg.REC16)  # whole tables: fine
        g.members[1].flow_partition(1, 2)
        with pytest.raises(rxg.RxgError, match="flow-partitioned"):
            g.rx_burst(frames, rxg.REC16)
        g.members[1].flow_partition(0, 1)
        g.rx_burst(frames, rxg.REC16)


def test_flow_partition_rejects_bad_arguments(engine):
    for part, n in ((0, 0), (3, 3), (0, rxg.RSS_RETA_SIZE + 1)):
        with pytest.raises(rxg.RxgError):
            engine.flow_partition(part, n)


@pytest.mark.parametrize("seed", [1, 2])
def test_flow_partition_replay_sequential_equivalence(seed):
    """Each RSS queue's burst + replay equals the reference loop run over that queue's packets
    in order, the table changing inside the burst (SYN -> child TCB, SYN_RECV -> ESTABLISHED,
    FIN -> CLOSED -> remove_tcb): the children's tuples hash to the queue of the SYN that made
    them, so the partitioned mirror holds them."""
    import ctypes as C

    from test_gpu_replay import Model, scenario, sequential_reference
    rows, frames = scenario(seed, n=1200)
    nparts = 2
    for p in range(nparts):
        mine = [f for f in frames if rxg.flow_part_of(f, nparts) == p]
        exp, ecnt, erows = sequential_reference(rows, mine)
        tcb, live = pktgen.table_arrays(rows)
        with rxg.Engine(device=0, max_batch=4096, max_bytes=8 << 20) as eng:
            eng.flow_partition(p, nparts)
            eng.tcb_load(tcb, live)
            eng.tcb_sync()
            eng.counters_reset()
            recs = eng.rx_burst(mine, rxg.REC16)
            model = Model(rows, eng)
            bufs = [C.create_string_buffer(f, max(len(f), 64)) for f in mine]
            addr = {C.addressof(b): i for i, b in enumerate(bufs)}
            got = [None] * len(mine)

            def free_mbuf(u, m):
                i = addr[m]
                if got[i] is None:
                    got[i] = ("free",)

            def rst(u, ip, tcp):
                got[addr[ip - 14]] = ("rst",)

            def tcpswitch(u, idx, st, tcp, ip, m):
                i = addr[m]
                got[i] = ("switch", idx, st)
                model.handle(idx, st, mine[i])
                return 0

            ops = rxg.HandoffOps(None, rxg.HANDOFF_FREE(free_mbuf), rxg.HANDOFF_ARP_IN(), rxg.HANDOFF_GET_MAC(),
                                 rxg.HANDOFF_ADD_MAC(), rxg.HANDOFF_SEND_RESET(rst), rxg.HANDOFF_ON_SEGMENT(),
                                 rxg.HANDOFF_TCPSWITCH(tcpswitch))
            ptrs = (C.c_void_p * len(bufs))(*[C.addressof(b) for b in bufs])
            lib = rxg.load_library()
            rc = lib.rxg_rx_replay(eng.ctx, C.byref(ops), ptrs, ptrs, recs.ctypes.data, len(bufs), 16)
            assert rc == 0, lib.rxg_last_error()
            for i, (v, idx, st) in enumerate(exp):
                if v == rxg.V_DISPATCH:
                    assert got[i] == ("switch", idx, st), (p, i, got[i], exp[i])
                elif v in (rxg.V_RST_NOPCB, rxg.V_RST_LISTEN_NONSYN):
                    assert got[i] == ("rst",), (p, i, got[i], exp[i])
            assert model.rows == erows
            assert eng.counters().tolist() == ecnt.tolist()


def _rss_tables():
    """T[i][v]: the RSS hash of 12 bytes holding v at position i (the hash is linear over
    GF(2), so a tuple's hash is the XOR of its bytes' entries)."""
    t = np.zeros((12, 256), dtype=np.uint32)
    for i in range(12):
        for v in range(256):
            w = bytearray(12)
            w[i] = v
            t[i, v] = rxg.rss_hash(bytes(w))
    return t


def test_flow_partitions_c5_full_size():
    """C5's scale (BASELINE.json configs[4]): 2^20 IMIX frames on 2^20 flows + a listener,
    two RSS queues.  Each queue's context holds about half the million tuples and classifies
    every frame steered to it to tcbs[1 + flow], ESTABLISHED, DISPATCH, both checksums 0."""
    n, flows, nparts = 1 << 20, 1 << 20, 2
    tcb, live = rxg.synthetic_tcb_table(flows)
    gen = rxg.Engine(device=0)
    parts = [rxg.Engine(device=0) for _ in range(nparts)]
    try:
        b = gen.synth(n=n, nflows=flows, mix=1, seed=0xF10, with_flows=True)
        gen.sync()
        fl = b["flow"].download(np.uint32, n)
        lens = b["len"].download(np.uint16, n)
        off = b["off64"].download(np.uint32, n)
        arena = b["arena"].download(np.uint8, b["arena_bytes"])
        # frame bytes 26..37 of every frame, then the queue by the byte tables
        pos = off.astype(np.int64)[:, None] * 64 + np.arange(26, 38)[None, :]
        w = arena[pos]
        t = _rss_tables()
        h = np.zeros(n, dtype=np.uint32)
        for i in range(12):
            h ^= t[i][w[:, i]]
        q = (h % rxg.RSS_RETA_SIZE) % nparts
        for k in range(0, n, 4099):  # spot-check the vectorised steering against the C ABI
            f = arena[int(off[k]) * 64:int(off[k]) * 64 + int(lens[k])].tobytes()
            assert rxg.flow_part_of(f, nparts) == q[k]
        keys = []
        for p, eng in enumerate(parts):
            eng.flow_partition(p, nparts)
            eng.tcb_load(tcb, live)
            eng.tcb_sync()
            keys.append(eng.tcb_keys())
            sel = np.nonzero(q == p)[0]
            m = len(sel)
            d_off = eng.to_device(off[sel].copy())
            d_len = eng.to_device(lens[sel].copy())
            out = eng.alloc(m * rxg.REC16)
            eng.counters_reset()
            eng.rx_burst_dev(b["arena"].ptr, d_off.ptr, d_len.ptr, m, out.ptr, rxg.REC16)
            eng.sync()
            rec = out.download(rxg.REC16_DTYPE, m)
            for a in (d_off, d_len, out):
                a.free()
            assert (rec["verdict"] == rxg.V_DISPATCH).all(), p
            assert (rec["tcb_idx"] == fl[sel].astype(np.int64) + 1).all(), p
            assert (rec["state"] == rxg.TCP_ESTABLISHED).all(), p
            assert (rec["ip_cksum"] == 0).all() and (rec["tcp_cksum"] == 0).all(), p
            assert (rec["datalen"] == lens[sel].astype(np.int64) - 54).all(), p
        assert sum(keys) == flows + 1 and min(keys) > 0.45 * flows, keys
    finally:
        for eng in parts:
            eng.close()
        gen.close()
