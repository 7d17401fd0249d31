"""GPU parity for the rx kernel's internal paths that small batches on a full grid never
reach:

* the per-wave LDS record ring filling up and flushing mid-stream (a wave sees more
  slices than the ring holds) -- forced with a one- or three-workgroup grid;
* runs of all-small slices (the prefetched small-slice pipeline) starting, continuing and
  ending next to class-path slices;
* the per-lane last-flow cache: a lane repeating its previous tuple (exact TCB, listener,
  no PCB, NULL slot before the listener) skips the probe and must give the same record.

Everything is compared bit-exact, records and counters, with the oracle.
"""
import random

import numpy as np
import pytest

import oracle
import pktgen
import rxg

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", params=[1, 3])
def small_grid_engine(request):
    """A context whose rx grid is `param` workgroups (rxg_config.max_blocks): 4 or 12 waves,
    so each wave walks many slices."""
    eng = rxg.Engine(device=0, max_batch=1 << 16, max_bytes=64 << 20, max_blocks=request.param)
    yield eng
    eng.close()


def _small_frame(rng, src, sport, dport, flags=0x10):
    # <= 64 bytes: 54 B of headers + 0..10 payload bytes
    return pktgen.frame(src_ip=src, sport=sport, dport=dport, flags=flags,
                        payload=rng.randbytes(rng.randrange(0, 11)))


def _batch(seed):
    """Stretches of slices (64 frames each) of three kinds, long enough that every wave of
    a 1- or 3-workgroup grid meets runs of each kind:
      'same'  : one tuple per lane repeated slice after slice (flow-cache hits), the tuple
                cycling through exact / listener / no-PCB / NULL-slot cases;
      'small' : random <= 64 B frames of random flows (cache misses, truncated frames);
      'mixed' : the random parity mixture (all size classes, malformed frames)."""
    rng = random.Random(seed)
    rows, flows, special = pktgen.parity_table(rng, 300)
    cases = [
        flows[3],                                        # exact hit
        (pktgen.ip4(10, 99, 1, 1), 7777, 80),            # listener :80, non-SYN -> RST
        (pktgen.ip4(10, 99, 1, 2), 7778, 8080),          # listener :8080 behind a NULL slot
        (pktgen.ip4(10, 99, 1, 3), 7779, 9999),          # no PCB -> RST
        special["dup"],                                  # duplicate tuple: lowest index
        special["hostdst"],                              # host-order dst: pass 1 misses
    ]
    frames = []
    plan = ["same"] * 24 + ["mixed"] * 8 + ["small"] * 20 + ["same"] * 16 + ["mixed"] * 4 + \
           ["small", "mixed"] * 10 + ["same"] * 40 + ["mixed"] * 12
    lane_case = [rng.randrange(len(cases)) for _ in range(64)]
    for kind in plan:
        if kind == "same":
            if rng.random() < 0.3:  # some lanes change flow between slices
                for _ in range(8):
                    lane_case[rng.randrange(64)] = rng.randrange(len(cases))
            for lane in range(64):
                src, sport, dport = cases[lane_case[lane]]
                flags = 0x02 if (lane % 5 == 0) else 0x10
                frames.append(_small_frame(rng, src, sport, dport, flags))
        elif kind == "small":
            for _ in range(64):
                src, sport, dport = rng.choice(flows)
                f = _small_frame(rng, src, sport, dport)
                if rng.random() < 0.1:
                    f = f[:rng.randrange(0, len(f) + 1)]  # truncated
                frames.append(f)
        else:
            frames.extend(pktgen.random_frame(rng, flows, special) for _ in range(64))
    return rows, frames


def _check(engine, rows, frames, rec_kind):
    arena, off, lens = pktgen.pack_arena(frames)
    tcb, live = pktgen.table_arrays(rows)
    engine.tcb_load(tcb, live)
    engine.counters_reset()
    got = engine.rx_arena(arena, off, lens, rec_kind)
    cnt = engine.counters()
    exp, ecnt = oracle.rx_batch(arena, off, lens, tcb, live)
    if rec_kind == rxg.REC16:
        exp = exp["c"]
    elif rec_kind == rxg.REC8:
        exp = rxg.rec8_pack(exp["c"])
    if got.tobytes() != exp.tobytes():
        g = got if rec_kind != rxg.REC48 else got["c"]
        e = exp if rec_kind != rxg.REC48 else exp["c"]
        gb = g.view(np.uint8).reshape(len(frames), -1)
        eb = e.view(np.uint8).reshape(len(frames), -1)
        bad = np.nonzero((gb != eb).any(axis=1))[0]
        i = int(bad[0])
        raise AssertionError(f"records differ at {len(bad)} frames, first {i} (slice {i // 64}, "
                             f"lane {i % 64}, len {len(frames[i])}): got {g[i]} exp {e[i]}")
    assert np.array_equal(cnt, ecnt), (cnt, ecnt)


@pytest.mark.parametrize("seed", [21, 22])
@pytest.mark.parametrize("rec_kind", [rxg.REC8, rxg.REC16, rxg.REC48])
def test_many_slices_per_wave(small_grid_engine, seed, rec_kind):
    rows, frames = _batch(seed)
    _check(small_grid_engine, rows, frames, rec_kind)


def test_partial_last_slice_after_small_run(small_grid_engine):
    """A run of full small slices followed by a partial last slice (n % 64 != 0): the run
    must stop before it (the partial slice takes the class path)."""
    rows, frames = _batch(23)
    frames = frames[:64 * 30 + 37]
    _check(small_grid_engine, rows, frames, rxg.REC48)
    _check(small_grid_engine, rows, frames, rxg.REC8)


# Size classes of the class path as (lowest, highest frame length, frames per
# round): the pipelined round loop must be right for every count of a class's frames in a
# slice -- one round, odd and even numbers of rounds, a last round partly filled.
_CLASSES = [(65, 128, 32), (129, 256, 16), (257, 512, 8), (513, 576, 8), (577, 768, 8),
            (769, 1024, 4), (1025, 1536, 4), (1537, 2048, 2)]


def _class_sweep_batch(seed):
    rng = random.Random(seed)
    rows, flows, special = pktgen.parity_table(rng, 200)
    frames = []
    for lo, hi, fpw in _CLASSES:
        counts = sorted({1, fpw - 1, fpw, fpw + 1, 2 * fpw, 2 * fpw + 1, 3 * fpw, 63, 64} - {0})
        for k in counts:
            k = min(k, 64)
            kinds = ["c"] * k + ["o"] * (64 - k)
            rng.shuffle(kinds)
            for kind in kinds:
                src, sport, dport = rng.choice(flows)
                if kind == "c":
                    n = rng.randrange(lo, hi + 1)
                else:  # the slice's other frames: small, or another class
                    n = rng.choice([rng.randrange(54, 65), rng.randrange(65, 1537)])
                f = pktgen.frame(src_ip=src, sport=sport, dport=dport, payload=rng.randbytes(max(0, n - 54)))
                if rng.random() < 0.05:  # a corrupted byte: checksums must say so
                    b = bytearray(f)
                    b[rng.randrange(14, len(b))] ^= 0x5A
                    f = bytes(b)
                frames.append(f)
    return rows, frames


@pytest.mark.parametrize("rec_kind", [rxg.REC8, rxg.REC16])
def test_class_round_counts(small_grid_engine, rec_kind):
    """Every streaming class with 1, FPW-1 .. 3*FPW, 63 and 64 frames in a slice: records
    and counters bit-exact with the oracle (the software-pipelined rounds)."""
    rows, frames = _class_sweep_batch(31)
    _check(small_grid_engine, rows, frames, rec_kind)


def test_class_round_counts_tx(small_grid_engine):
    """tx generate over the same slices: equal to the oracle's checksums byte for byte."""
    rows, frames = _class_sweep_batch(32)
    arena, off, lens = pktgen.pack_arena(frames)
    got = small_grid_engine.tx_arena(arena, off, lens)
    exp = oracle.tx_batch(arena, off, lens)
    assert got.tobytes() == exp.tobytes()


@pytest.mark.parametrize("by_ref", [False, True])
@pytest.mark.parametrize("rec_kind", [rxg.REC8, rxg.REC16, rxg.REC48])
def test_many_slices_per_wave_fused(small_grid_engine, rec_kind, by_ref):
    """The fused payload hand-off (rxg_rx_burst_payload_dev) over the same many-slices-per-wave
    batches: the copy form, and the by-reference form whose record ring also stages the
    messages, here flushing mid-stream from both the all-small and the class
    path -- records, counters and every message bit-exact with the oracle, every payload's
    bytes where its message points."""
    from oracle import payload as opl
    rows, frames = _batch(24)
    tcb, live = pktgen.table_arrays(rows)
    eng = small_grid_engine
    eng.tcb_load(tcb, live)
    eng.counters_reset()
    recs, pay, msgs, (arena, off, lens) = eng.rx_burst_payload(frames, rec_kind, by_reference=by_ref)
    cnt = eng.counters()
    exp, ecnt = oracle.rx_batch(arena, off, lens, tcb, live)
    want = exp if rec_kind == rxg.REC48 else exp["c"] if rec_kind == rxg.REC16 else rxg.rec8_pack(exp["c"])
    assert recs.tobytes() == want.tobytes()
    assert np.array_equal(cnt, ecnt), (cnt, ecnt)
    e_msgs, pays = opl.slots(frames, exp["c"], off)
    for name in ("arena_off", "len", "flags"):
        bad = np.nonzero(msgs[name] != e_msgs[name])[0]
        assert len(bad) == 0, f"msgs.{name} differs at {len(bad)} frames, first {bad[:1]}"
    assert (msgs["len"] > 0).sum() > 1000
    for i, p in enumerate(pays):
        if p is not None:
            o = int(msgs[i]["arena_off"])
            assert pay[o:o + len(p)].tobytes() == p, f"frame {i}: payload bytes differ"
