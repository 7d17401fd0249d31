"""GPU parity over launch grids whose last generation of slices is partial (HISTORY.md §9,
"Launch tail").

A launch deals its slices round-robin over the waves of its grid (rxg_config.max_blocks caps
it).  These tests pick grids for which the last generation holds a half, a third or a quarter
of the waves (the shapes for which experiment variant 52 cuts that generation into 2, 3 or 4
pieces per slice), with a partial last slice, REC8/16/48, multi-burst launches, tx and short
bursts, and compare everything bit-exact with the oracle.  The production kernel deals whole
slices; the helper below reproduces the experiment's piece count only to choose the grids.
"""
import random

import numpy as np
import pytest

import oracle
import pktgen
import rxg

pytestmark = pytest.mark.gpu


def pieces(nslices: int, blocks: int) -> int:
    """Experiment variant 52's piece count g (rxg_kernels.hip BurstCursor::units_init) for a grid of `blocks`."""
    nwaves = 4 * blocks
    full = (nslices // nwaves) * nwaves
    tail = nslices - full
    return 1 if tail == 0 else max(1, min(nwaves // tail, 4))


def grid_for(nslices: int, g: int) -> int:
    for b in range(1, 4096):
        if (nslices + 3) // 4 >= b and pieces(nslices, b) == g:
            return b
    raise AssertionError(f"no grid gives {g} pieces for {nslices} slices")


def test_piece_formula_cases():
    # the configurations DESIGN.md quotes: 2^20 frames on 768 workgroups -> 3 pieces of 22
    assert pieces(16384, 768) == 3
    assert pieces(1, 1) == 4 and pieces(2, 1) == 2 and pieces(3, 1) == 1
    assert pieces(144, 7) == 4 and pieces(144, 11) == 3 and pieces(144, 15) == 2


@pytest.fixture(scope="module")
def batch():
    rows, frames = pktgen.parity_set(seed=4242, n=64 * 143 + 37)  # 144 slices, the last partial
    return rows, frames


def _expect(rows, frames, kind):
    arena, off, lens = pktgen.pack_arena(frames)
    tcb, live = pktgen.table_arrays(rows)
    exp, ecnt = oracle.rx_batch(arena, off, lens, tcb, live)
    if kind == rxg.REC16:
        exp = exp["c"]
    elif kind == rxg.REC8:
        exp = rxg.rec8_pack(exp["c"])
    return arena, off, lens, tcb, live, exp, ecnt


@pytest.mark.parametrize("g", [2, 3, 4])
@pytest.mark.parametrize("kind", [rxg.REC8, rxg.REC16, rxg.REC48])
def test_pieces_single_burst(batch, g, kind):
    rows, frames = batch
    nslices = (len(frames) + 63) // 64
    blocks = grid_for(nslices, g)
    arena, off, lens, tcb, live, exp, ecnt = _expect(rows, frames, kind)
    with rxg.Engine(device=0, max_batch=1 << 15, max_bytes=32 << 20, max_blocks=blocks) as eng:
        eng.tcb_load(tcb, live)
        eng.counters_reset()
        got = eng.rx_arena(arena, off, lens, kind)
        cnt = eng.counters()
    if got.tobytes() != exp.tobytes():
        gb = got.view(np.uint8).reshape(len(frames), -1)
        eb = exp.view(np.uint8).reshape(len(frames), -1)
        bad = np.nonzero((gb != eb).any(axis=1))[0]
        raise AssertionError(f"g={g} blocks={blocks}: {len(bad)} records differ, first frame {bad[0]}")
    assert cnt.tolist() == ecnt.tolist()


@pytest.mark.parametrize("g", [2, 3, 4])
def test_pieces_multi_burst(batch, g):
    """Several bursts of one pool in one launch: pieces of the last generation may fall in
    any burst, and a piece past a burst's last frame holds nothing."""
    rows, frames = batch
    rng = random.Random(g)
    n = len(frames)
    cuts = [0] + sorted(rng.sample(range(1, n), 6)) + [n]
    nslices = sum((cuts[j + 1] - cuts[j] + 63) // 64 for j in range(len(cuts) - 1))
    blocks = grid_for(nslices, g)
    kind = rxg.REC8
    arena, off, lens, tcb, live, exp, ecnt = _expect(rows, frames, kind)
    with rxg.Engine(device=0, max_batch=1 << 15, max_bytes=32 << 20, max_blocks=blocks) as eng:
        eng.tcb_load(tcb, live)
        d_arena = eng.to_device(arena)
        dev, bursts = [], []
        try:
            for j in range(len(cuts) - 1):
                a, b = cuts[j], cuts[j + 1]
                do, dl, dout = eng.to_device(off[a:b]), eng.to_device(lens[a:b]), eng.alloc((b - a) * kind)
                dev += [do, dl, dout]
                bursts.append((do.ptr, dl.ptr, b - a, dout.ptr))
            eng.counters_reset()
            eng.rx_bursts_dev(d_arena.ptr, bursts, kind)
            eng.sync()
            cnt = eng.counters()
            got = np.concatenate([dev[3 * j + 2].download(rxg.rec_dtype(kind), cuts[j + 1] - cuts[j])
                                  for j in range(len(cuts) - 1)])
        finally:
            for d in dev + [d_arena]:
                d.free()
    assert got.tobytes() == exp.tobytes()
    assert cnt.tolist() == ecnt.tolist()


@pytest.mark.parametrize("g", [2, 3, 4])
def test_pieces_tx(batch, g):
    rows, frames = batch
    nslices = (len(frames) + 63) // 64
    blocks = grid_for(nslices, g)
    arena, off, lens = pktgen.pack_arena(frames)
    with rxg.Engine(device=0, max_batch=1 << 15, max_bytes=32 << 20, max_blocks=blocks) as eng:
        got = eng.tx_arena(arena, off, lens)
    assert got.tobytes() == oracle.tx_batch(arena, off, lens).tobytes()


@pytest.mark.parametrize("n", [1, 5, 17, 32, 63, 64, 65, 100, 200])
def test_small_bursts_pieces(n):
    """Bursts of a few slices: one workgroup, fewer slices than waves; the reference's own
    burst is MAX_PKT_BURST = 32 (main.c:116)."""
    rows, frames = pktgen.parity_set(seed=900 + n, n=n)
    arena, off, lens, tcb, live, exp, ecnt = _expect(rows, frames, rxg.REC16)
    with rxg.Engine(device=0, max_batch=1 << 12, max_bytes=8 << 20) as eng:
        eng.tcb_load(tcb, live)
        eng.counters_reset()
        got = eng.rx_arena(arena, off, lens, rxg.REC16)
        cnt = eng.counters()
    assert got.tobytes() == exp.tobytes()
    assert cnt.tolist() == ecnt.tolist()


@pytest.mark.parametrize("kind", [rxg.REC8, rxg.REC16])
def test_deep_pipeline_multi_burst(kind):
    """A launch with >= 16 slices per wave (rxg_kernels.hip kDeepSlicesPerWave) runs the
    two-deep all-small pipeline: one workgroup (4 waves) over ~150 slices in 7 bursts, runs of
    64 B slices between mixed ones, bit-exact with the oracle."""
    rng = random.Random(77)
    rows, frames = pktgen.parity_set(seed=4343, n=64 * 143 + 37)
    # long runs of <= 64 B frames so all-small runs of several slices occur per wave
    for start in (0, 2048, 5000):
        for i in range(start, start + 1500):
            src, sport, dport = rng.choice([(0x0A000001, 1024, 80), (0x0A000002, 1025, 80)])
            frames[i] = pktgen.frame(src_ip=src, sport=sport, dport=dport, payload=bytes(rng.randrange(0, 11)))
    n = len(frames)
    cuts = [0] + sorted(rng.sample(range(1, n), 6)) + [n]
    arena, off, lens, tcb, live, exp, ecnt = _expect(rows, frames, kind)
    with rxg.Engine(device=0, max_batch=1 << 15, max_bytes=32 << 20, max_blocks=1) as eng:
        eng.tcb_load(tcb, live)
        d_arena = eng.to_device(arena)
        dev, bursts = [], []
        try:
            for j in range(len(cuts) - 1):
                a, b = cuts[j], cuts[j + 1]
                do, dl, dout = eng.to_device(off[a:b]), eng.to_device(lens[a:b]), eng.alloc((b - a) * kind)
                dev += [do, dl, dout]
                bursts.append((do.ptr, dl.ptr, b - a, dout.ptr))
            eng.counters_reset()
            eng.rx_bursts_dev(d_arena.ptr, bursts, kind)
            eng.sync()
            cnt = eng.counters()
            got = np.concatenate([dev[3 * j + 2].download(rxg.rec_dtype(kind), cuts[j + 1] - cuts[j])
                                  for j in range(len(cuts) - 1)])
            single = eng.rx_arena(arena, off, lens, kind)  # one burst: also >= 16 slices per wave
        finally:
            for d in dev + [d_arena]:
                d.free()
    assert got.tobytes() == exp.tobytes()
    assert single.tobytes() == exp.tobytes()
    assert cnt.tolist() == ecnt.tolist()
