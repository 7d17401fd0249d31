"""GPU: fixed-stride bursts (rxg_rx_bursts_strided_dev): frame i of a
burst at 64-byte slot slot0 + i * stride64 of the pool, no offset list.  Records and counters
equal the oracle's and the list form's (rxg_rx_bursts_dev with off64[i] = slot0 + i *
stride64) for every record kind, several bursts per launch, the C2 configuration at full size,
the payload gather and the replay with its fix-ups on the GPU (which read the burst's offsets
through a list the library writes)."""
import numpy as np
import pytest

import oracle
import pktgen
import rxg
import test_gpu_replay
from test_gpu_parity import assert_records_equal

pytestmark = pytest.mark.gpu


def pack_strided(frames, stride64, slot0=0):
    """frames at slots slot0 + i * stride64 (each at most 64 * stride64 bytes); the slack
    holds garbage the kernel must ignore."""
    n = len(frames)
    assert all(len(f) <= 64 * stride64 for f in frames)
    arena = np.full(max((slot0 + n * stride64) * 64, 64), 0xA5, dtype=np.uint8)
    for i, f in enumerate(frames):
        o = (slot0 + i * stride64) * 64
        arena[o:o + len(f)] = np.frombuffer(f, dtype=np.uint8)
    lens = np.array([len(f) for f in frames], dtype=np.uint16)
    off = (slot0 + np.arange(n, dtype=np.uint64) * stride64).astype(np.uint32)
    return arena, off, lens


def _free(*ds):
    for d in ds:
        d.free()


@pytest.mark.parametrize("rec", [rxg.REC8, rxg.REC16, rxg.REC48])
def test_strided_equals_oracle_and_list_form(engine, rec):
    rows, frames = pktgen.parity_set(seed=600 + rec, n=5000)
    stride = (max(len(f) for f in frames) + 63) // 64
    tcb, live = pktgen.table_arrays(rows)
    engine.tcb_load(tcb, live)
    # three bursts of one pool: ragged sizes, partial slices, a one-frame burst
    cuts = [0, 1, 2048 + 17, 5000]
    arena, off, lens = pack_strided(frames, stride, slot0=3)
    da, do, dl = engine.to_device(arena), engine.to_device(off), engine.to_device(lens)
    n = len(frames)
    out_s, out_l = engine.alloc(n * rec), engine.alloc(n * rec)
    try:
        engine.counters_reset()
        engine.rx_bursts_strided_dev(da.ptr, stride, [(3 + cuts[j] * stride, dl.ptr + 2 * cuts[j], cuts[j + 1] - cuts[j],
                                                       out_s.ptr + rec * cuts[j]) for j in range(3)], rec)
        engine.sync()
        cnt_s = engine.counters()
        engine.counters_reset()
        engine.rx_bursts_dev(da.ptr, [(do.ptr + 4 * cuts[j], dl.ptr + 2 * cuts[j], cuts[j + 1] - cuts[j],
                                       out_l.ptr + rec * cuts[j]) for j in range(3)], rec)
        engine.sync()
        assert out_s.download(np.uint8, n * rec).tobytes() == out_l.download(np.uint8, n * rec).tobytes()
        assert cnt_s.tolist() == engine.counters().tolist()
        exp, ecnt = oracle.rx_batch(arena, off, lens, tcb, live)
        assert cnt_s.tolist() == ecnt.tolist()
        got = out_s.download(rxg.rec_dtype(rec), n)
        if rec == rxg.REC48:
            assert_records_equal(got, exp, frames)
        elif rec == rxg.REC16:
            assert got.tobytes() == exp["c"].tobytes()
        else:
            assert got.tobytes() == rxg.rec8_pack(exp["c"]).tobytes()
    finally:
        _free(da, do, dl, out_s, out_l)


def test_strided_c2_full_size(engine):
    """C2 (BASELINE configs[1]: 2^20 x 64 B, one flow): the synthetic pool puts frame i at
    slot i, so the strided form (stride 1) reads the same frames without off64[]."""
    n = 1 << 20
    dev = engine.synth(n=n, nflows=1, len_a=64, seed=612)
    tcb, live = rxg.synthetic_tcb_table(1)
    engine.tcb_load(tcb, live)
    off = dev["off64"].download(np.uint32, n)
    assert (off == np.arange(n, dtype=np.uint32)).all()
    a, b = engine.alloc(n * 8), engine.alloc(n * 8)
    try:
        engine.counters_reset()
        engine.rx_bursts_strided_dev(dev["arena"].ptr, 1, [(0, dev["len"].ptr, n, a.ptr)], rxg.REC8)
        engine.sync()
        c1 = engine.counters()
        engine.counters_reset()
        engine.rx_burst_dev(dev["arena"].ptr, dev["off64"].ptr, dev["len"].ptr, n, b.ptr, rxg.REC8)
        engine.sync()
        assert a.download(np.uint8, n * 8).tobytes() == b.download(np.uint8, n * 8).tobytes()
        assert c1.tolist() == engine.counters().tolist()
        assert int(c1[rxg.COUNTERS.index("dispatch")]) == n and int(c1[rxg.COUNTERS.index("tcp_cksum_bad")]) == 0
        # sixteen bursts of one 1 GiB pool (the multi-burst leg), strided
        pool = engine.synth(n=16 * n, nflows=1, len_a=64, seed=613)
        big = engine.alloc(16 * n * 8)
        try:
            engine.counters_reset()
            engine.rx_bursts_strided_dev(pool["arena"].ptr, 1, [(j * n, pool["len"].ptr + 2 * j * n, n, big.ptr + 8 * j * n)
                                                                for j in range(16)], rxg.REC8)
            engine.sync()
            c = engine.counters()
            assert int(c[0]) == 16 * n and int(c[rxg.COUNTERS.index("dispatch")]) == 16 * n
            tail = rxg.rec8_expand(big.download(rxg.REC8_DTYPE, 4096, offset_bytes=(16 * n - 4096) * 8))
            assert (tail["tcb_idx"] == 1).all() and (tail["verdict"] == rxg.V_DISPATCH).all()
        finally:
            big.free()
            for v in pool.values():
                if isinstance(v, rxg.DevArray):
                    v.free()
    finally:
        _free(a, b)
        for v in dev.values():
            if isinstance(v, rxg.DevArray):
                v.free()


def test_strided_payload_gather(engine):
    """The gather after a strided burst reads the frames through the offsets the library
    writes for it: the same arena and descriptors as after the list form."""
    rows, frames = pktgen.parity_set(seed=620, n=3000)
    stride = (max(len(f) for f in frames) + 63) // 64
    tcb, live = pktgen.table_arrays(rows)
    engine.tcb_load(tcb, live)
    engine.arp_disable()
    arena, off, lens = pack_strided(frames, stride)
    da, do, dl = engine.to_device(arena), engine.to_device(off), engine.to_device(lens)
    n = len(frames)
    out = engine.alloc(n * 16)
    try:
        engine.rx_burst_dev(da.ptr, do.ptr, dl.ptr, n, out.ptr, rxg.REC16)
        engine.sync()
        ga, gm, gu = engine.payload_gather(n, 1 << 24)
        ga, gm = ga.copy(), gm.copy()
        engine.rx_bursts_strided_dev(da.ptr, stride, [(0, dl.ptr, n, out.ptr)], rxg.REC16)
        engine.sync()
        sa, sm, su = engine.payload_gather(n, 1 << 24)
        assert su == gu and sm.tobytes() == gm.tobytes() and sa[:gu].tobytes() == ga[:gu].tobytes()
        assert gu > 0
    finally:
        _free(da, do, dl, out)


@pytest.mark.parametrize("seed", [1, 2])
def test_strided_replay_fixups_on_device(seed):
    """test_gpu_replay's sequential-equivalence scenario with the burst strided and every
    fix-up a GPU re-classification (RXG_CFG_REPLAY_ON_DEVICE), which reads the strided burst's
    frames through the library-written offsets."""
    eng = rxg.Engine(device=0, max_batch=1 << 16, max_bytes=64 << 20, flags=rxg.CFG_REPLAY_ON_DEVICE)
    keep = []

    def burst(e, frames):
        stride = (max(len(f) for f in frames) + 63) // 64
        arena, off, lens = pack_strided(frames, stride)
        da, dl = e.to_device(arena), e.to_device(lens)
        out = e.alloc(len(frames) * 16)
        keep.extend([da, dl, out])
        e.rx_bursts_strided_dev(da.ptr, stride, [(0, dl.ptr, len(frames), out.ptr)], rxg.REC16)
        e.sync()
        return out.download(rxg.REC16_DTYPE, len(frames))

    try:
        test_gpu_replay.run_replay_equivalence(eng, seed, burst)
        assert eng.replay_stats()["device_launches"] > 0
    finally:
        _free(*keep)
        eng.close()


def test_strided_rejects_bad_arguments(engine):
    import ctypes as C
    lib = rxg.load_library()
    d = engine.alloc(1024)
    try:
        one = (rxg.DevStridedBurst * 1)(rxg.DevStridedBurst(d.ptr, 4, 0, d.ptr))
        assert lib.rxg_rx_bursts_strided_dev(engine.ctx, d.ptr, 0, one, 1, rxg.REC8, None) == -22  # stride 0
        big = (rxg.DevStridedBurst * 1)(rxg.DevStridedBurst(d.ptr, 4, 0xFFFFFFF0, d.ptr))
        assert lib.rxg_rx_bursts_strided_dev(engine.ctx, d.ptr, 8, big, 1, rxg.REC8, None) == -22  # slot overflow
        nul = (rxg.DevStridedBurst * 1)(rxg.DevStridedBurst(None, 4, 0, d.ptr))
        assert lib.rxg_rx_bursts_strided_dev(engine.ctx, d.ptr, 1, nul, 1, rxg.REC8, None) == -22
        assert lib.rxg_rx_bursts_strided_dev(engine.ctx, d.ptr, 1, one, 1, 7, None) == -22  # record kind
        assert lib.rxg_rx_bursts_strided_dev(engine.ctx, d.ptr, 1, None, 1, rxg.REC8, None) == -22
        assert C.sizeof(rxg.DevStridedBurst) == 24
    finally:
        d.free()
