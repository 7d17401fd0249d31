"""GPU: zero-copy batches (include/rxg.h rxg_host_register): frames, descriptors and records
in host memory that the kernels read and write over PCIe.  Results equal the device-resident
path and the oracle; tx generate rewrites the host frames in place."""
import numpy as np
import pytest

import oracle
import pktgen
import rxg
from test_gpu_parity import assert_records_equal

pytestmark = pytest.mark.gpu


def _aligned(nbytes, align=4096):
    raw = np.zeros(nbytes + align, dtype=np.uint8)
    o = (-raw.ctypes.data) % align
    return raw[o:o + nbytes]


def test_rx_and_tx_on_registered_host_memory(engine):
    rows, frames = pktgen.parity_set(seed=31, n=3000)
    arena, off, lens = pktgen.pack_arena(frames)
    tcb, live = pktgen.table_arrays(rows)
    engine.tcb_load(tcb, live)
    n = len(lens)
    h_arena = _aligned(arena.nbytes + 64)
    h_arena[: arena.nbytes] = arena
    h_off, h_len = _aligned(n * 4), _aligned(n * 2)
    h_off[:] = off.view(np.uint8)
    h_len[:] = lens.view(np.uint8)
    h_out = _aligned(n * 48)
    regs = [h_arena, h_off, h_len, h_out]
    dev = [engine.host_register(a) for a in regs]
    try:
        engine.rx_burst_dev(dev[0], dev[1], dev[2], n, dev[3], rxg.REC48)
        engine.sync()
        got = h_out.view(rxg.REC48_DTYPE).copy()
        exp, _ = oracle.rx_batch(arena, off, lens, tcb, live)
        assert_records_equal(got, exp, frames)
        assert got.tobytes() == engine.rx_arena(arena, off, lens, rxg.REC48).tobytes()
        # tx generate in place on the host frames
        engine.tx_cksum_dev(dev[0], dev[1], dev[2], n)
        engine.sync()
        assert np.array_equal(h_arena[: arena.nbytes], oracle.tx_batch(arena, off, lens))
    finally:
        for a in regs:
            engine.host_unregister(a)


def test_register_rejects_bad_arguments(engine):
    lib = rxg.load_library()
    import ctypes as C
    d = C.c_void_p()
    assert lib.rxg_host_register(engine.ctx, None, 64, C.byref(d)) < 0
    assert lib.rxg_host_unregister(engine.ctx, None) < 0
