"""GPU parity at BASELINE.json's full sizes (C2, C3, C4: 2^20 frames per launch, the bench's
own synthetic batches), through properties that do not depend on the oracle's speed:
  - every frame's record against the generator's ground truth (flow f -> tcbs[1 + f],
    ESTABLISHED, DISPATCH, both checksums valid, datalen = len - 54);
  - the counters against the batch (rx, bytes, dispatch, exact hits);
  - a seeded random sample of 4 096 frames bit-exact against the oracle (REC48), frames
    downloaded from the same device arena;
  - tx generate over the whole batch with both checksum fields first zeroed reproduces the
    arena byte for byte (the synthetic frames carry valid checksums)."""
import numpy as np
import pytest

import oracle
import rxg
from test_gpu_parity import assert_records_equal

pytestmark = pytest.mark.gpu
N = 1 << 20
CONFIGS = {  # name: (frame_len, flows, mix) as bench.py's WORKLOADS
    "c2_64B_1flow": (64, 1, 0),
    "c3_1500B_1Kflows": (1500, 1000, 0),
    "c4_imix_64Kflows": (0, 65536, 1),
}


@pytest.fixture(scope="module", params=sorted(CONFIGS))
def batch(engine, request):
    L, flows, mix = CONFIGS[request.param]
    b = engine.synth(n=N, nflows=flows, len_a=L or 1500, mix=mix, seed=0xF0115, with_flows=True)
    engine.sync()
    tcb, live = rxg.synthetic_tcb_table(flows)
    b["tcb"], b["live"], b["name"] = tcb, live, request.param
    yield b
    for v in b.values():
        if isinstance(v, rxg.DevArray):
            v.free()


@pytest.mark.parametrize("kind", [rxg.REC16, rxg.REC8])
def test_full_size_records_and_counters(engine, batch, kind):
    """REC8 (the bench's records) is checked through its rxg_rec16 view (rxg_rec8_expand):
    every field, and both checksums as 0 (valid)."""
    engine.tcb_load(batch["tcb"], batch["live"])
    engine.counters_reset()
    out = engine.alloc(N * kind)
    try:
        engine.rx_burst_dev(batch["arena"].ptr, batch["off64"].ptr, batch["len"].ptr, N, out.ptr, kind)
        engine.sync()
        rec = out.download(rxg.rec_dtype(kind), N)
    finally:
        out.free()
    if kind == rxg.REC8:
        rec = rxg.rec8_expand(rec)
    flow = batch["flow"].download(np.uint32, N)
    lens = batch["len"].download(np.uint16, N).astype(np.int64)
    assert (rec["verdict"] == rxg.V_DISPATCH).all()
    assert (rec["tcb_idx"] == (flow.astype(np.int64) + 1)).all()
    assert (rec["state"] == rxg.TCP_ESTABLISHED).all()
    assert (rec["ip_cksum"] == 0).all() and (rec["tcp_cksum"] == 0).all()
    assert (rec["flags"] == (rxg.F_IP_OK | rxg.F_TCP_OK)).all()
    assert (rec["tcp_flags"] == 0x10).all()
    assert (rec["datalen"] == lens - 54).all()
    c = dict(zip(rxg.COUNTERS, engine.counters().tolist()))
    assert c["rx"] == N and c["dispatch"] == N and c["tcb_hit_exact"] == N
    assert c["bytes"] == int(lens.sum()) and c["tcp_cksum_bad"] == 0 and c["ip_cksum_bad"] == 0


def _sample(batch, k=4096, seed=5):
    rng = np.random.default_rng(seed)
    idx = np.sort(rng.choice(N, size=k, replace=False))
    off = batch["off64"].download(np.uint32, N)[idx]
    lens = batch["len"].download(np.uint16, N)[idx]
    frames = [batch["arena"].download(np.uint8, int(l), offset_bytes=int(o) * 64).tobytes()
              for o, l in zip(off, lens)]
    return idx, frames


def test_full_size_sample_matches_oracle(engine, batch):
    engine.tcb_load(batch["tcb"], batch["live"])
    out = engine.alloc(N * rxg.REC48)
    try:
        engine.rx_burst_dev(batch["arena"].ptr, batch["off64"].ptr, batch["len"].ptr, N, out.ptr, rxg.REC48)
        engine.sync()
        rec = out.download(rxg.REC48_DTYPE, N)
    finally:
        out.free()
    idx, frames = _sample(batch)
    arena, off, lens = rxg.pack_arena(frames)
    exp, _ = oracle.rx_batch(arena, off, lens, batch["tcb"], batch["live"])
    assert_records_equal(np.ascontiguousarray(rec[idx]), exp, frames)


def test_full_size_tx_regenerates_checksums(engine, batch):
    """rx_kernel<0> over the whole batch with the two checksum fields zeroed (ip_out sums
    them as zero, ip.c:104-118) writes back exactly the synthetic frames' checksums."""
    nbytes = batch["arena_bytes"]
    ref = batch["arena"].download(np.uint8, nbytes)
    off = batch["off64"].download(np.uint32, N).astype(np.int64) * 64
    lens = batch["len"].download(np.uint16, N)
    zeroed = ref.copy()
    for b in (24, 25, 50, 51):
        zeroed[off + b] = 0
    work = engine.to_device(zeroed)
    try:
        engine.tx_cksum_dev(work.ptr, batch["off64"].ptr, batch["len"].ptr, N)
        engine.sync()
        got = work.download(np.uint8, nbytes)
    finally:
        work.free()
    assert (lens >= 54).all()
    assert np.array_equal(got, ref)
