"""GPU parity for BASELINE.json configs[4] ("C5"): bidirectional -- tx checksum generate
(ip_out, tcp_ip_stack/ip.c:97-118) and rx parse + verify + classify (findtcb,
tcp_tcb.c:127-173) -- over 2^20 IMIX frames (64/576/1500 at 7:4:1) against a table of
2^20 flows + 1 listener (1 048 577 TCBs, 52x the reference's TOTAL_TCBS).

* rx, whole batch, by property: every frame DISPATCH to tcbs[1 + flow], ESTABLISHED, both
  checksums 0, datalen = len - 54; counters equal the batch.
* rx, a seeded 512-frame sample bit-exact against the oracle's linear two-pass findtcb over
  the full 1 M-entry table (REC48: every extracted field).
* tx, whole batch: the checksum fields zeroed, rxg_tx_cksum_dev regenerates the arena byte
  for byte -- device-resident, and in the zero-copy form bench.py's C5 leg uses (frames,
  descriptors in pinned host memory read and patched in place over PCIe).
* tx -> rx: the regenerated host frames, copied in, verify to 0x0000 and classify as above.
"""
import numpy as np
import pytest

import oracle
import rxg
from test_gpu_parity import assert_records_equal

pytestmark = pytest.mark.gpu
N = 1 << 20
FLOWS = 1 << 20


@pytest.fixture(scope="module")
def c5(engine):
    b = engine.synth(n=N, nflows=FLOWS, mix=1, seed=0xC5C5, with_flows=True)
    engine.sync()
    tcb, live = rxg.synthetic_tcb_table(FLOWS)
    engine.tcb_load(tcb, live)
    engine.tcb_sync()
    b["tcb"], b["live"] = tcb, live
    b["flows"] = b["flow"].download(np.uint32, N)
    b["lens"] = b["len"].download(np.uint16, N)
    b["off"] = b["off64"].download(np.uint32, N)
    b["ref"] = b["arena"].download(np.uint8, b["arena_bytes"])
    yield b
    for v in b.values():
        if isinstance(v, rxg.DevArray):
            v.free()


def _rx_property(engine, b, arena_ptr, off_ptr, len_ptr):
    engine.counters_reset()
    out = engine.alloc(N * rxg.REC16)
    try:
        engine.rx_burst_dev(arena_ptr, off_ptr, len_ptr, N, out.ptr, rxg.REC16)
        engine.sync()
        rec = out.download(rxg.REC16_DTYPE, N)
    finally:
        out.free()
    lens = b["lens"].astype(np.int64)
    assert (rec["verdict"] == rxg.V_DISPATCH).all()
    assert (rec["tcb_idx"] == b["flows"].astype(np.int64) + 1).all()
    assert (rec["state"] == rxg.TCP_ESTABLISHED).all()
    assert (rec["ip_cksum"] == 0).all() and (rec["tcp_cksum"] == 0).all()
    assert (rec["datalen"] == lens - 54).all()
    c = dict(zip(rxg.COUNTERS, engine.counters().tolist()))
    assert c["rx"] == N and c["dispatch"] == N and c["tcb_hit_exact"] == N and c["bytes"] == int(lens.sum())
    assert c["ip_cksum_bad"] == 0 and c["tcp_cksum_bad"] == 0


def test_c5_rx_whole_batch(engine, c5):
    assert set(np.unique(c5["lens"]).tolist()) == {64, 576, 1500}
    assert len(np.unique(c5["flows"])) > 600_000   # most of the million flows are hit
    _rx_property(engine, c5, c5["arena"].ptr, c5["off64"].ptr, c5["len"].ptr)


def test_c5_rx_sample_matches_oracle(engine, c5):
    out = engine.alloc(N * rxg.REC48)
    try:
        engine.rx_burst_dev(c5["arena"].ptr, c5["off64"].ptr, c5["len"].ptr, N, out.ptr, rxg.REC48)
        engine.sync()
        rec = out.download(rxg.REC48_DTYPE, N)
    finally:
        out.free()
    rng = np.random.default_rng(55)
    idx = np.sort(rng.choice(N, size=512, replace=False))
    frames = [c5["ref"][int(o) * 64:int(o) * 64 + int(l)].tobytes() for o, l in zip(c5["off"][idx], c5["lens"][idx])]
    arena, off, lens = rxg.pack_arena(frames)
    exp, _ = oracle.rx_batch(arena, off, lens, c5["tcb"], c5["live"])
    assert_records_equal(np.ascontiguousarray(rec[idx]), exp, frames)


def _zeroed(c5):
    z = c5["ref"].copy()
    o = c5["off"].astype(np.int64) * 64
    for b in (24, 25, 50, 51):
        z[o + b] = 0
    return z


def test_c5_tx_regenerates_device_resident(engine, c5):
    work = engine.to_device(_zeroed(c5))
    try:
        engine.tx_cksum_dev(work.ptr, c5["off64"].ptr, c5["len"].ptr, N)
        engine.sync()
        assert np.array_equal(work.download(np.uint8, c5["arena_bytes"]), c5["ref"])
    finally:
        work.free()


def test_c5_tx_zero_copy_then_rx(engine, c5):
    """bench.py's C5 tx direction: host frames and descriptors in pinned memory, the kernel
    reads them over PCIe and patches each frame's first line in place; then the rx
    direction copies the regenerated frames in and verifies/classifies them."""
    nb = c5["arena_bytes"]
    h_tx, h_off, h_len = engine.pinned(nb), engine.pinned(N * 4), engine.pinned(N * 2)
    try:
        h_tx.np[:nb] = _zeroed(c5)
        h_off.np[: N * 4] = c5["off"].view(np.uint8)
        h_len.np[: N * 2] = c5["lens"].view(np.uint8)
        engine.tx_cksum_dev(h_tx.ptr, h_off.ptr, h_len.ptr, N)
        engine.sync()
        assert np.array_equal(h_tx.np[:nb], c5["ref"])
        d = engine.alloc(nb)
        try:
            engine.h2d(d.ptr, h_tx.ptr, nb)
            engine.sync()
            _rx_property(engine, c5, d.ptr, c5["off64"].ptr, c5["len"].ptr)
        finally:
            d.free()
    finally:
        for a in (h_tx, h_off, h_len):
            a.free()
