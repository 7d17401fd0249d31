"""GPU: the incremental device TCB mirror (csrc/rxg_mirror.h) under live churn, and the
ordering of mirror writes against bursts on other streams.

* Churn: a 65 537-TCB table (the C4 flow count) takes rounds of the writes the reference
  makes -- tcp_listen appending children (tcp_states.c:150-207), remove_tcb NULLing slots
  (tcp_tcb.c:175-186), tuple rewrites (tcp_states.c:25-27), state changes, listeners coming
  and going -- each applied as O(1) device patches, never a reload.  After every round a
  burst is compared bit-exact (REC48 + counters) with the oracle's findtcb over the table as
  it stands.
* Ordering: a long burst on a caller stream is still running when the table changes; it must
  classify against the old table, and the next burst (same stream, another stream, or the
  context's) against the new one, with no host synchronisation in between.
"""
import random

import numpy as np
import pytest
import torch

import oracle
import pktgen
import rxg

pytestmark = pytest.mark.gpu
DST = pktgen.ip4(192, 168, 78, 2)
DST_RAW = pktgen.raw_of_host(DST)


def _frames(rng, rows, n):
    """Frames aimed at live flows, dead flows, never-seen flows and listeners."""
    out = []
    for _ in range(n):
        k = rng.random()
        if k < 0.6:
            r = rows[rng.randrange(len(rows))]
            if r is None or r[1] < 0 or r[1] > 65535 or r[0] < 0 or r[0] > 65535:
                r = (80, 1024, DST_RAW, pktgen.ip4(10, 0, 0, 1), 4)
            out.append(pktgen.frame(src_ip=r[3], dst_ip=DST, sport=r[1], dport=r[0],
                                    flags=rng.choice([0x10, 0x18, 0x02, 0x11])))
        elif k < 0.85:
            out.append(pktgen.frame(src_ip=pktgen.ip4(172, 16, rng.randrange(256), rng.randrange(256)),
                                    dst_ip=DST, sport=rng.randrange(1024, 65536),
                                    dport=rng.choice([80, 80, 8080, 9000]), flags=rng.choice([0x02, 0x10])))
        else:
            out.append(pktgen.frame(src_ip=pktgen.ip4(10, 0, rng.randrange(256), rng.randrange(256)),
                                    dst_ip=DST, sport=1024 + rng.randrange(64511), dport=80, flags=0x10))
    return out


def _check_burst(eng, rows, frames):
    tcb, live = pktgen.table_arrays(rows)
    arena, off, lens = pktgen.pack_arena(frames)
    eng.counters_reset()
    got = eng.rx_arena(arena, off, lens, rxg.REC48)
    cnt = eng.counters()
    exp, ecnt = oracle.rx_batch(arena, off, lens, tcb, live)
    if got.tobytes() != exp.tobytes():
        bad = np.nonzero(got.view(np.uint8).reshape(len(frames), 48) != exp.view(np.uint8).reshape(len(frames), 48))[0]
        i = int(bad[0])
        raise AssertionError(f"{len(set(bad.tolist()))} records differ; first {i}: {got[i]} vs {exp[i]}")
    assert cnt.tolist() == ecnt.tolist()


def test_churn_incremental_mirror_equals_oracle(engine):
    rng = random.Random(2024)
    nflows = 65536
    t0, l0 = rxg.synthetic_tcb_table(nflows)
    rows = [(int(t["dport"]), int(t["sport"]), int(t["ipv4_dst"]), int(t["ipv4_src"]), int(t["state"]))
            for t in t0]
    engine.tcb_load(t0, l0)
    engine.tcb_sync()
    for rnd in range(12):
        for _ in range(rng.choice([1, 8, 64, 300])):
            k = rng.random()
            n = len(rows)
            if k < 0.35:    # tcp_listen: a child at Ntcb (sometimes a duplicate tuple: SYN resent)
                src = pktgen.ip4(172, 16, rng.randrange(256), rng.randrange(256))
                r = (80, rng.randrange(1024, 65536), DST_RAW, src, rng.choice([3, 4]))
                if rng.random() < 0.1:
                    live_rows = [x for x in rows[1:200] if x is not None]
                    r = live_rows[rng.randrange(len(live_rows))][:4] + (3,)
                rows.append(r)
                engine.tcb_upsert(n, *r)
            elif k < 0.6:   # remove_tcb
                i = rng.randrange(n)
                if rows[i] is not None:
                    rows[i] = None
                    engine.tcb_remove(i)
            elif k < 0.75:  # tuple rewrite of a live slot (tcp_syn_sent) or reuse of a NULL slot
                i = rng.randrange(1, n)
                r = (rng.choice([80, 8080, 9000]), rng.randrange(1024, 65536), DST_RAW,
                     pktgen.ip4(10, 9, rng.randrange(256), rng.randrange(256)), rng.randrange(7))
                rows[i] = r
                engine.tcb_upsert(i, *r)
            else:           # state change, listeners included
                i = rng.randrange(n)
                if rows[i] is not None:
                    st = rng.choice([0, 1, 3, 4, 5, 6])
                    rows[i] = rows[i][:4] + (st,)
                    engine.tcb_set_state(i, st)
        _check_burst(engine, rows, _frames(rng, rows, 3000))
    # the patched table equals a fresh full build of the same rows
    tcb, live = pktgen.table_arrays(rows)
    frames = _frames(rng, rows, 3000)
    arena, off, lens = pktgen.pack_arena(frames)
    a = engine.rx_arena(arena, off, lens, rxg.REC48)
    engine.tcb_load(tcb, live)
    b = engine.rx_arena(arena, off, lens, rxg.REC48)
    assert a.tobytes() == b.tobytes()


@pytest.mark.parametrize("second", ["same", "other", "ctx"])
def test_mirror_write_between_bursts_on_caller_streams(engine, second):
    """a mirror write must neither reach a burst still running on a caller stream
    nor be missed by the next burst, without the caller synchronising."""
    n, nflows = 1 << 20, 1000
    dev = engine.synth(n=n, nflows=nflows, len_a=1500, seed=77, with_flows=True)
    t0, l0 = rxg.synthetic_tcb_table(nflows)
    engine.tcb_load(t0, l0)
    engine.tcb_sync()
    engine.sync()
    flows = dev["flow"].download(np.uint32, n)
    out_a, out_b = engine.alloc(n * 16), engine.alloc(n * 16)
    s1 = torch.cuda.Stream()
    s2 = torch.cuda.Stream()
    try:
        for _ in range(3):  # a few rounds: the first burst is long (≈250 us), the writes are µs
            engine.tcb_load(t0, l0)
            engine.tcb_sync()
            engine.sync()
            torch.cuda.synchronize()
            engine.rx_burst_dev(dev["arena"].ptr, dev["off64"].ptr, dev["len"].ptr, n, out_a.ptr, 16,
                                s1.cuda_stream)
            removed = list(range(1, nflows + 1, 3))
            for i in removed:       # flows 0, 3, 6, ... lose their TCB
                engine.tcb_remove(i)
            stream_b = {"same": s1.cuda_stream, "other": s2.cuda_stream, "ctx": None}[second]
            engine.rx_burst_dev(dev["arena"].ptr, dev["off64"].ptr, dev["len"].ptr, n, out_b.ptr, 16, stream_b)
            torch.cuda.synchronize()
            engine.sync()
            a = out_a.download(rxg.REC16_DTYPE, n)
            b = out_b.download(rxg.REC16_DTYPE, n)
            assert (a["tcb_idx"] == flows.astype(np.int32) + 1).all()
            assert (a["verdict"] == rxg.V_DISPATCH).all()
            gone = (flows % 3) == 0
            assert (b["tcb_idx"][~gone] == flows[~gone].astype(np.int32) + 1).all()
            # a removed flow falls to the listener (slot 0) as a non-SYN: reset (tcp_in.c:54-59)
            assert (b["tcb_idx"][gone] == 0).all() and (b["verdict"][gone] == rxg.V_RST_LISTEN_NONSYN).all()
    finally:
        for d in (out_a, out_b):
            d.free()
        for v in dev.values():
            if isinstance(v, rxg.DevArray):
                v.free()


@pytest.mark.parametrize("lazy", [False, True])
def test_mirror_write_waits_for_every_reader_stream(lazy):
    """a long burst on s1, then a short one on s2, then removals, then a burst on
    the context's stream, with no host synchronisation in between.  The removals must wait
    for BOTH readers (one entry per reader stream, csrc/rxg_host.cpp order_table_reader_after;
    lazy = RXG_CFG_STREAMS_OUTLIVE_WRITES: the events recorded on the reader streams when the
    write is pushed, wait_table_readers): the s1 burst classifies every frame against the old
    table."""
    engine = rxg.Engine(device=0, max_batch=1 << 16, max_bytes=64 << 20,
                        flags=rxg.CFG_STREAMS_OUTLIVE_WRITES if lazy else 0)
    n, nflows, m = 1 << 20, 1000, 4096
    dev = engine.synth(n=n, nflows=nflows, len_a=1500, seed=78, with_flows=True)
    t0, l0 = rxg.synthetic_tcb_table(nflows)
    flows = dev["flow"].download(np.uint32, n)
    out_a, out_s, out_c = engine.alloc(n * 16), engine.alloc(m * 16), engine.alloc(n * 16)
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    for st in (s1, s2):  # required in the lazy mode, harmless otherwise
        engine.stream_register(st.cuda_stream)
    try:
        for _ in range(3):
            engine.tcb_load(t0, l0)
            engine.tcb_sync()
            engine.sync()
            torch.cuda.synchronize()
            engine.rx_burst_dev(dev["arena"].ptr, dev["off64"].ptr, dev["len"].ptr, n, out_a.ptr, 16, s1.cuda_stream)
            engine.rx_burst_dev(dev["arena"].ptr, dev["off64"].ptr, dev["len"].ptr, m, out_s.ptr, 16, s2.cuda_stream)
            for i in range(1, nflows + 1, 2):   # flows 0, 2, 4, ... lose their TCB
                engine.tcb_remove(i)
            engine.rx_burst_dev(dev["arena"].ptr, dev["off64"].ptr, dev["len"].ptr, n, out_c.ptr, 16, None)
            torch.cuda.synchronize()
            engine.sync()
            a = out_a.download(rxg.REC16_DTYPE, n)
            s = out_s.download(rxg.REC16_DTYPE, m)
            c = out_c.download(rxg.REC16_DTYPE, n)
            assert (a["tcb_idx"] == flows.astype(np.int32) + 1).all(), "the s1 burst saw the removals"
            assert (s["tcb_idx"] == flows[:m].astype(np.int32) + 1).all()
            gone = (flows % 2) == 0
            assert (c["tcb_idx"][~gone] == flows[~gone].astype(np.int32) + 1).all()
            assert (c["tcb_idx"][gone] == 0).all() and (c["verdict"][gone] == rxg.V_RST_LISTEN_NONSYN).all()
    finally:
        for d in (out_a, out_s, out_c):
            d.free()
        for v in dev.values():
            if isinstance(v, rxg.DevArray):
                v.free()
        engine.close()


@pytest.mark.parametrize("lazy", [False, True])
def test_caller_stream_destroyed_before_the_next_write(lazy):
    """rxg.h: a caller stream that ran a burst may be destroyed before the context's next table
    write: once synchronised without RXG_CFG_STREAMS_OUTLIVE_WRITES, once retired
    (rxg_stream_retire) with it.  The write and the next bursts still succeed and classify
    against the new table.  With the flag, a launch on an unregistered stream is refused with
    -EINVAL and launches nothing (round 3 crashed in tcb_sync: an event recorded on a stream
    destroyed before the write, gpurun_out/r03s3l/pytest_mirror.txt)."""
    import ctypes as C
    # the HIP runtime this process already runs (librxg's and torch's), by its loaded path
    path = next(ln.split()[-1] for ln in open("/proc/self/maps") if "libamdhip64.so" in ln)
    hip = C.CDLL(path)
    engine = rxg.Engine(device=0, max_batch=1 << 16, max_bytes=64 << 20,
                        flags=rxg.CFG_STREAMS_OUTLIVE_WRITES if lazy else 0)
    n, nflows = 1 << 16, 64
    dev = engine.synth(n=n, nflows=nflows, len_a=64, seed=79, with_flows=True)
    t0, l0 = rxg.synthetic_tcb_table(nflows)
    flows = dev["flow"].download(np.uint32, n)
    out = engine.alloc(n * 16)
    try:
        engine.tcb_load(t0, l0)
        engine.tcb_sync()
        for rep in range(3):
            st = C.c_void_p()
            assert hip.hipStreamCreate(C.byref(st)) == 0
            if lazy:
                with pytest.raises(rxg.RxgError, match="not registered"):
                    engine.rx_burst_dev(dev["arena"].ptr, dev["off64"].ptr, dev["len"].ptr, n, out.ptr, 16, st.value)
            engine.stream_register(st.value)
            engine.rx_burst_dev(dev["arena"].ptr, dev["off64"].ptr, dev["len"].ptr, n, out.ptr, 16, st.value)
            if lazy:
                engine.stream_retire(st.value)   # before the synchronisation: the order is taken now
            assert hip.hipStreamSynchronize(st) == 0
            if not lazy:
                engine.stream_retire(st.value)   # accepted either way
            assert hip.hipStreamDestroy(st) == 0
            a = out.download(rxg.REC16_DTYPE, n)
            live = np.ones(nflows, dtype=bool)
            live[: 2 * rep] = False
            assert (a["tcb_idx"][live[flows]] == flows[live[flows]].astype(np.int32) + 1).all()
            engine.tcb_remove(2 * rep + 1)       # flow 2 rep loses its TCB: a write
            engine.tcb_remove(2 * rep + 2)
            engine.tcb_sync()
            engine.rx_burst_dev(dev["arena"].ptr, dev["off64"].ptr, dev["len"].ptr, n, out.ptr, 16, None)
            engine.sync()
            c = out.download(rxg.REC16_DTYPE, n)
            gone = flows < 2 * rep + 2
            assert (c["tcb_idx"][~gone] == flows[~gone].astype(np.int32) + 1).all()
            assert (c["tcb_idx"][gone] == 0).all()
    finally:
        out.free()
        for v in dev.values():
            if isinstance(v, rxg.DevArray):
                v.free()
        engine.close()


def test_rejected_launch_keeps_the_previous_burst_replayable():
    """under RXG_CFG_STREAMS_OUTLIVE_WRITES a launch on an unregistered stream
    is refused before anything changes (no mirror sync, replay state kept), so rxg_rx_replay
    of the burst before it still runs, and calls the hand-off for every dispatched packet."""
    import ctypes as C
    import pktgen
    path = next(ln.split()[-1] for ln in open("/proc/self/maps") if "libamdhip64.so" in ln)
    hip = C.CDLL(path)
    engine = rxg.Engine(device=0, max_batch=4096, max_bytes=8 << 20, flags=rxg.CFG_STREAMS_OUTLIVE_WRITES)
    rows, frames = pktgen.parity_set(11, 600)
    dev = engine.synth(n=256, nflows=4, len_a=64, seed=80)
    out = engine.alloc(256 * 16)
    st = C.c_void_p()
    assert hip.hipStreamCreate(C.byref(st)) == 0
    try:
        tcb, live = pktgen.table_arrays(rows)
        engine.tcb_load(tcb, live)
        engine.arp_disable()
        recs = engine.rx_burst(frames, rxg.REC16)
        with pytest.raises(rxg.RxgError, match="not registered"):
            engine.rx_burst_dev(dev["arena"].ptr, dev["off64"].ptr, dev["len"].ptr, 256, out.ptr, 16, st.value)
        seen = []

        def tcpswitch(u, idx, state, tcp, ip, m):
            seen.append(idx)
            return 0
        ops = rxg.HandoffOps(None, rxg.HANDOFF_FREE(), rxg.HANDOFF_ARP_IN(), rxg.HANDOFF_GET_MAC(),
                             rxg.HANDOFF_ADD_MAC(), rxg.HANDOFF_SEND_RESET(), rxg.HANDOFF_ON_SEGMENT(),
                             rxg.HANDOFF_TCPSWITCH(tcpswitch))
        bufs = [C.create_string_buffer(f, max(len(f), 64)) for f in frames]
        ptrs = (C.c_void_p * len(bufs))(*[C.addressof(b) for b in bufs])
        lib = rxg.load_library()
        assert lib.rxg_rx_replay(engine.ctx, C.byref(ops), ptrs, ptrs, recs.ctypes.data, len(bufs), 16) == 0
        disp = recs["tcb_idx"][recs["verdict"] == rxg.V_DISPATCH]
        assert seen == disp.tolist() and len(seen) > 100
    finally:
        assert hip.hipStreamDestroy(st) == 0
        out.free()
        for v in dev.values():
            if isinstance(v, rxg.DevArray):
                v.free()
        engine.close()


def test_carried_patches_then_a_burst_on_another_stream(engine):
    """A few writes (a list the next burst on the context's stream carries itself, DESIGN.md
    §2.1), that burst, then at once a burst on a caller stream: the second must see the new
    table, though no patch launch ran -- it waits for the event recorded after the carrying
    burst when it is needed (mirror_event) -- and so must a third on the context's stream."""
    n, nflows = 1 << 16, 1000
    dev = engine.synth(n=n, nflows=nflows, len_a=576, seed=91, with_flows=True)
    t0, l0 = rxg.synthetic_tcb_table(nflows)
    flows = dev["flow"].download(np.uint32, n)
    outs = [engine.alloc(n * 16) for _ in range(3)]
    s2 = torch.cuda.Stream()
    try:
        for rnd in range(3):
            engine.tcb_load(t0, l0)
            engine.tcb_sync()
            engine.sync()
            torch.cuda.synchronize()
            removed = set(range(1 + rnd, nflows + 1, 97))  # ~10 removals: a carried list
            for i in sorted(removed):
                engine.tcb_remove(i)
            engine.rx_burst_dev(dev["arena"].ptr, dev["off64"].ptr, dev["len"].ptr, n, outs[0].ptr, 16, None)
            engine.rx_burst_dev(dev["arena"].ptr, dev["off64"].ptr, dev["len"].ptr, n, outs[1].ptr, 16,
                                s2.cuda_stream)
            engine.rx_burst_dev(dev["arena"].ptr, dev["off64"].ptr, dev["len"].ptr, n, outs[2].ptr, 16, None)
            torch.cuda.synchronize()
            engine.sync()
            gone = np.isin(flows.astype(np.int64) + 1, sorted(removed))
            for o in outs:
                r = o.download(rxg.REC16_DTYPE, n)
                assert (r["tcb_idx"][~gone] == flows[~gone].astype(np.int32) + 1).all()
                assert (r["tcb_idx"][gone] == 0).all() and (r["verdict"][gone] == rxg.V_RST_LISTEN_NONSYN).all()
    finally:
        for d in outs:
            d.free()
        for v in dev.values():
            if isinstance(v, rxg.DevArray):
                v.free()


@pytest.mark.parametrize("reader", ["stream", "server"])
@pytest.mark.parametrize("narp", [300, 250])
def test_carried_list_then_an_overflowing_arp_list(reader, narp):
    """a TCB list the burst on the context's stream carries, then an ARP list
    that does not fit beside it (narp alone past kLaunchPatchMax = 256, or the sum past it)
    and so goes through its own patch launch before that burst.  The next table reader -- a
    burst on a caller stream, or a served burst (rxg_server_burst_dev) -- must wait for the
    carrying burst, not for the event recorded after the ARP launch (csrc/rxg_host.cpp
    launch_patch_list: the event stays stale while a list is still to be carried).  A long
    burst on the context's stream runs first, so the ARP launch, the carrying burst and the
    reader all queue behind it.  Checked against the synthetic flows and the oracle's ARP set
    (arp.c:282-317: a learned source is no longer flagged)."""
    eng = rxg.Engine(device=0)
    n, nflows, m = 1 << 20, 1000, 4096
    dev = eng.synth(n=n, nflows=nflows, len_a=1500, seed=606, with_flows=True)
    t0, l0 = rxg.synthetic_tcb_table(nflows)
    srcs = t0["ipv4_src"][1:]
    flows = dev["flow"].download(np.uint32, n)
    out_a, out_b, out_r = eng.alloc(n * 16), eng.alloc(n * 16), eng.alloc(n * 16)
    s2 = torch.cuda.Stream()
    # never-seen addresses fill the ARP list past the join's room; the flows' own sources
    # (half of them) are learned in the same list
    extra = [pktgen.ip4(100, 64, i >> 8, i & 255) for i in range(narp - nflows // 2 if narp > nflows // 2 else 0)]
    try:
        if reader == "server":
            eng.server_start(rxg.REC16, blocks=4, max_frames=m)
        for rnd in range(3):
            eng.tcb_load(t0, l0)
            eng.arp_load([pktgen.ip4(99, 0, i >> 8, i & 255) for i in range(1200)])  # sized: no rebuild below
            eng.rx_burst_dev(dev["arena"].ptr, dev["off64"].ptr, dev["len"].ptr, m, out_r.ptr, 16, None)
            eng.sync()
            torch.cuda.synchronize()
            eng.rx_burst_dev(dev["arena"].ptr, dev["off64"].ptr, dev["len"].ptr, n, out_a.ptr, 16, None)  # long
            removed = sorted(set(range(1 + rnd, nflows + 1, 97)))  # ~10 removals: a carried list
            for i in removed:
                eng.tcb_remove(i)
            learned = [int(x) for x in srcs[rnd % 2::2][:min(narp, nflows // 2)]] + extra
            learned = learned[:narp]
            for ip in learned:
                eng.arp_learned(ip)
            eng.rx_burst_dev(dev["arena"].ptr, dev["off64"].ptr, dev["len"].ptr, n, out_b.ptr, 16, None)  # carries
            if reader == "stream":
                eng.rx_burst_dev(dev["arena"].ptr, dev["off64"].ptr, dev["len"].ptr, n, out_r.ptr, 16, s2.cuda_stream)
                k = n
            else:
                eng.server_burst_dev(dev["arena"].ptr, dev["off64"].ptr, dev["len"].ptr, m, out_r.ptr, rxg.REC16)
                k = m
            torch.cuda.synchronize()
            eng.sync()
            gone = np.isin(flows.astype(np.int64) + 1, removed)
            known = np.isin(srcs[flows], np.asarray(learned, dtype=srcs.dtype))
            a = out_a.download(rxg.REC16_DTYPE, n)
            assert (a["tcb_idx"] == flows.astype(np.int32) + 1).all(), "the first burst saw later writes"
            for o, kk in ((out_b, n), (out_r, k)):
                r = o.download(rxg.REC16_DTYPE, kk)
                g, kn, f = gone[:kk], known[:kk], flows[:kk]
                assert (r["tcb_idx"][~g] == f[~g].astype(np.int32) + 1).all(), (rnd, "stale TCB entry")
                assert (r["tcb_idx"][g] == 0).all() and (r["verdict"][g] == rxg.V_RST_LISTEN_NONSYN).all(), rnd
                assert ((r["flags"] & rxg.F_ARP_LEARN) != 0).tolist() == (~kn).tolist(), (rnd, "stale ARP entry")
        if reader == "server":
            eng.server_stop()
    finally:
        for d in (out_a, out_b, out_r):
            d.free()
        for v in dev.values():
            if isinstance(v, rxg.DevArray):
                v.free()
        eng.close()


@pytest.mark.parametrize("lazy", [False, True])
def test_counters_read_waits_for_caller_stream_bursts(lazy):
    """rxg_counters_read is synchronous for every burst of the context, on whatever stream it
    was launched (include/rxg.h): long bursts on two caller streams, then at once a read with
    no synchronisation by the caller -- it counts every frame of both (the counter block is
    the reference's tcp_in counters, tcp_in.c:18-19, merged per context)."""
    engine = rxg.Engine(device=0, flags=rxg.CFG_STREAMS_OUTLIVE_WRITES if lazy else 0)
    n, nflows = 1 << 20, 1000
    dev = engine.synth(n=n, nflows=nflows, len_a=1500, seed=707, with_flows=True)
    t0, l0 = rxg.synthetic_tcb_table(nflows)
    out1, out2 = engine.alloc(n * 8), engine.alloc(n * 8)
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    for st in (s1, s2):
        engine.stream_register(st.cuda_stream)
    try:
        engine.tcb_load(t0, l0)
        engine.tcb_sync()
        engine.sync()
        for rnd in range(3):
            engine.counters_reset()
            engine.sync()
            torch.cuda.synchronize()
            engine.rx_burst_dev(dev["arena"].ptr, dev["off64"].ptr, dev["len"].ptr, n, out1.ptr, 8, s1.cuda_stream)
            engine.rx_burst_dev(dev["arena"].ptr, dev["off64"].ptr, dev["len"].ptr, n, out2.ptr, 8, s2.cuda_stream)
            cnt = dict(zip(rxg.COUNTERS, engine.counters().tolist()))
            assert cnt["rx"] == 2 * n and cnt["dispatch"] == 2 * n and cnt["tcb_hit_exact"] == 2 * n, (rnd, cnt)
            assert cnt["bytes"] == 2 * n * 1500
        torch.cuda.synchronize()
    finally:
        for d in (out1, out2):
            d.free()
        for v in dev.values():
            if isinstance(v, rxg.DevArray):
                v.free()
        engine.close()
