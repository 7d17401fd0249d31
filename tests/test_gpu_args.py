"""GPU: launches with misaligned device buffers are refused (-EINVAL, with the reason)
before anything runs: the rx kernel reads descriptors as u32 / u16 and frames in 16-byte
chunks, and stores each slice's records with 8- or 16-byte vector stores."""
import ctypes as C

import numpy as np
import pytest

import pktgen
import rxg

pytestmark = pytest.mark.gpu


def test_misaligned_buffers_are_refused(engine):
    frames = [pktgen.frame(sport=4000 + i, payload=bytes(i % 7)) for i in range(100)]
    arena, off, lens = pktgen.pack_arena(frames)
    lib = rxg.load_library()
    da, do, dl = engine.to_device(arena), engine.to_device(off), engine.to_device(lens)
    dout = engine.alloc(len(frames) * 48 + 64)
    try:
        n = len(frames)
        for frames_p, off_p, len_p, out_p, kind, why in [
            (da.ptr + 8, do.ptr, dl.ptr, dout.ptr, rxg.REC16, b"frame pool"),
            (da.ptr, do.ptr + 2, dl.ptr, dout.ptr, rxg.REC16, b"alignment"),
            (da.ptr, do.ptr, dl.ptr + 1, dout.ptr, rxg.REC16, b"alignment"),
            (da.ptr, do.ptr, dl.ptr, dout.ptr + 8, rxg.REC16, b"alignment"),
            (da.ptr, do.ptr, dl.ptr, dout.ptr + 4, rxg.REC8, b"alignment"),
        ]:
            b = rxg.DevBatch(frames_p, off_p, len_p, n, kind, out_p)
            assert lib.rxg_rx_burst_dev(engine.ctx, C.byref(b), None) == -22
            assert why in lib.rxg_last_error()
        # 8-byte aligned records are fine for REC8, and the burst still equals the oracle's
        got = engine.rx_arena(arena, off, lens, rxg.REC8)
        b = rxg.DevBatch(da.ptr, do.ptr, dl.ptr, n, rxg.REC8, dout.ptr + 8)
        assert lib.rxg_rx_burst_dev(engine.ctx, C.byref(b), None) == 0
        engine.sync()
        assert dout.download(rxg.REC8_DTYPE, n, offset_bytes=8).tobytes() == got.tobytes()
        # tx: the same rules for its frames and descriptors
        t = rxg.DevTxBatch(da.ptr + 4, do.ptr, dl.ptr, n)
        assert lib.rxg_tx_cksum_dev(engine.ctx, C.byref(t), None) == -22
    finally:
        for d in (da, do, dl, dout):
            d.free()


def test_replay_refused_after_a_rejected_launch(engine):
    """a launch refused at validation (misaligned records) leaves nothing to
    replay; a replay whose n matches the previous, good burst is refused, not replayed from
    that burst's records."""
    frames = [pktgen.frame(sport=5000 + i) for i in range(64)]
    arena, off, lens = pktgen.pack_arena(frames)
    lib = rxg.load_library()
    da, do, dl = engine.to_device(arena), engine.to_device(off), engine.to_device(lens)
    dout = engine.alloc(len(frames) * 16 + 64)
    try:
        n = len(frames)
        good = rxg.DevBatch(da.ptr, do.ptr, dl.ptr, n, rxg.REC16, dout.ptr)
        assert lib.rxg_rx_burst_dev(engine.ctx, C.byref(good), None) == 0
        engine.sync()
        recs = dout.download(rxg.REC16_DTYPE, n)
        ops = rxg.HandoffOps()
        bufs = [C.create_string_buffer(f, 64) for f in frames]
        ptrs = (C.c_void_p * n)(*[C.addressof(b) for b in bufs])
        assert lib.rxg_rx_replay(engine.ctx, C.byref(ops), ptrs, ptrs, recs.ctypes.data, n, 16) == 0
        bad = rxg.DevBatch(da.ptr, do.ptr, dl.ptr, n, rxg.REC16, dout.ptr + 8)
        assert lib.rxg_rx_burst_dev(engine.ctx, C.byref(bad), None) == -22
        assert lib.rxg_rx_replay(engine.ctx, C.byref(ops), ptrs, ptrs, recs.ctypes.data, n, 16) == -22
        assert b"failed" in lib.rxg_last_error()
    finally:
        for d in (da, do, dl, dout):
            d.free()
