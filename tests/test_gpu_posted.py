"""GPU: tcbs[] writes posted from other threads (rxg_tcb_post) take effect at the next
burst, in posting order, and the burst equals the oracle run on the resulting table."""
import threading

import numpy as np
import pytest

import oracle
import pktgen
import rxg

pytestmark = pytest.mark.gpu


def test_posted_writes_apply_at_the_next_burst(engine):
    dst = pktgen.ip4(192, 168, 78, 2)
    raw_dst = pktgen.raw_of_host(dst)
    nthreads, per = 4, 300
    n = 1 + nthreads * per
    # the rx thread's own table: the listener only
    tcb, live = pktgen.table_arrays([(80, 0, raw_dst, 0, pktgen.LISTENING)])
    engine.tcb_load(tcb, live)
    engine.tcb_sync()

    def app(t):  # an application thread: alloc_tcb + socket_bind-style tuple writes
        for i in range(per):
            idx = 1 + t * per + i
            src = pktgen.ip4(10, 50, t, i & 255) + ((i >> 8) << 8)
            assert engine.tcb_post_upsert(idx, 80, 2000 + i, raw_dst, src, pktgen.ESTABLISHED, idx) == 0
            if i % 50 == 0:  # state changes and removals, in the thread's order
                assert engine.tcb_post_set_state(idx, 3) == 0
            if i % 97 == 0:
                assert engine.tcb_post_remove(idx) == 0

    ths = [threading.Thread(target=app, args=(t,)) for t in range(nthreads)]
    for th in ths:
        th.start()
    for th in ths:
        th.join()
    assert engine.tcb_count() == 1  # nothing applied before the rx thread's next burst

    rows = [(80, 0, raw_dst, 0, pktgen.LISTENING)] + [None] * (n - 1)
    frames = []
    for t in range(nthreads):
        for i in range(per):
            idx = 1 + t * per + i
            src = pktgen.ip4(10, 50, t, i & 255) + ((i >> 8) << 8)
            st = 3 if i % 50 == 0 else pktgen.ESTABLISHED
            rows[idx] = None if i % 97 == 0 else (80, 2000 + i, raw_dst, src, st)
            frames.append(pktgen.frame(src_ip=src, sport=2000 + i, dport=80))
    arena, off, lens = pktgen.pack_arena(frames)
    engine.counters_reset()
    got = engine.rx_arena(arena, off, lens, rxg.REC48)  # the burst drains the queue first
    assert engine.tcb_count() == n
    etcb, elive = pktgen.table_arrays(rows)
    exp, ecnt = oracle.rx_batch(arena, off, lens, etcb, elive)
    assert got.tobytes() == exp.tobytes()
    assert np.array_equal(engine.counters(), ecnt)


def test_post_rejects_bad_kind_and_drain_reports_errors(engine):
    import ctypes as C
    bad = rxg.TcbOp(7, 1)
    assert rxg.load_library().rxg_tcb_post(engine.ctx, C.byref(bad)) < 0
    engine.tcb_load(*pktgen.table_arrays([(80, 0, 0, 0, pktgen.LISTENING)]))
    assert engine.tcb_post_set_state(5, 4) == 0  # slot 5 does not exist: fails when applied
    assert engine.tcb_post_upsert(2, 81, 1, 2, 3, pktgen.ESTABLISHED) == 0
    with pytest.raises(rxg.RxgError):
        engine.tcb_drain()
    assert engine.tcb_count() == 3  # the later write was still applied
