"""GPU soak (opt-in: RXG_SOAK=<seconds>): random parity batches over random launch shapes,
compared bit-exact with the oracle until the time budget is spent.

Each case draws a seed, a batch (the parity mixture of tests/pktgen.py: every size class,
malformed frames, listeners, NULL slots, duplicate tuples, host-order dst), runs of <= 64 B
frames of a few flows (the all-small path and its flow cache), a grid (rxg_config.max_blocks
1..40: one to many slices per wave, so both the one- and the two-deep all-small pipelines
run), a record kind, and single- or multi-burst launch.  Skipped unless RXG_SOAK is set: the
round's regular GPU suite covers each path once; this is for hunting rare interleavings.
"""
import os
import random
import time

import numpy as np
import pytest

import oracle
import pktgen
import rxg

pytestmark = pytest.mark.gpu
BUDGET = float(os.environ.get("RXG_SOAK", "0"))


@pytest.mark.skipif(BUDGET <= 0, reason="opt-in soak: set RXG_SOAK=<seconds>")
def test_soak_random_launch_shapes():
    t_end = time.time() + BUDGET
    master = random.Random(int(os.environ.get("RXG_SOAK_SEED", "2026")))
    engines = {}
    cases = 0
    try:
        while time.time() < t_end:
            seed = master.randrange(1 << 30)
            rng = random.Random(seed)
            n = rng.choice([1, 31, 64, 65, 200, 1000, 4096, 9000])
            rows, frames = pktgen.parity_set(seed=seed, n=n, nflows=rng.choice([3, 50, 400]))
            for _ in range(rng.randrange(0, 4)):  # runs of small frames of a few flows
                a = rng.randrange(0, n)
                for i in range(a, min(n, a + rng.randrange(64, 700))):
                    frames[i] = pktgen.frame(src_ip=0x0A000001 + (i % 3), sport=1024 + (i % 3), dport=80,
                                             payload=bytes(rng.randrange(0, 11)))
            kind = rng.choice([rxg.REC8, rxg.REC16, rxg.REC48])
            blocks = rng.choice([1, 2, 3, 5, 8, 13, 40])
            if blocks not in engines:
                engines[blocks] = rxg.Engine(device=0, max_batch=1 << 14, max_bytes=32 << 20, max_blocks=blocks)
            eng = engines[blocks]
            arena, off, lens = pktgen.pack_arena(frames)
            tcb, live = pktgen.table_arrays(rows)
            exp, ecnt = oracle.rx_batch(arena, off, lens, tcb, live)
            if kind == rxg.REC16:
                exp = exp["c"]
            elif kind == rxg.REC8:
                exp = rxg.rec8_pack(exp["c"])
            eng.tcb_load(tcb, live)
            eng.counters_reset()
            multi = n > 2 and rng.random() < 0.5
            if not multi:
                got = eng.rx_arena(arena, off, lens, kind)
            else:
                k = rng.randrange(2, min(n, 33))
                cuts = [0] + sorted(rng.sample(range(1, n), k - 1)) + [n]
                d_arena = eng.to_device(arena)
                dev, bursts = [], []
                try:
                    for j in range(k):
                        lo, hi = cuts[j], cuts[j + 1]
                        do, dl = eng.to_device(off[lo:hi]), eng.to_device(lens[lo:hi])
                        dout = eng.alloc((hi - lo) * kind)
                        dev += [do, dl, dout]
                        bursts.append((do.ptr, dl.ptr, hi - lo, dout.ptr))
                    eng.rx_bursts_dev(d_arena.ptr, bursts, kind)
                    eng.sync()
                    got = np.concatenate([dev[3 * j + 2].download(rxg.rec_dtype(kind), cuts[j + 1] - cuts[j])
                                          for j in range(k)])
                finally:
                    for d in dev + [d_arena]:
                        d.free()
            cnt = eng.counters()
            assert got.tobytes() == exp.tobytes(), \
                f"seed {seed} n {n} kind {kind} blocks {blocks} multi {multi}: records differ"
            assert cnt.tolist() == ecnt.tolist(), f"seed {seed}: counters differ"
            cases += 1
            if cases % 50 == 0:
                print(f"soak: {cases} cases", flush=True)  # progress (run with -s)
    finally:
        for e in engines.values():
            e.close()
    print(f"soak: {cases} cases bit-exact")
    assert cases > 0


@pytest.mark.skipif(BUDGET <= 0, reason="opt-in soak: set RXG_SOAK=<seconds>")
def test_soak_served_bursts():
    """The latency-mode server under random requests (round 4's forms: descriptors in the
    mailbox, partial all-small slices, one or two slices shared by the workgroup's waves,
    per-wave counters): random parity batches cut into host bursts of 1..300 frames, served
    by servers of 1 / 3 / 8 workgroups in every placement, each burst equal to the oracle's
    records; counters equal the oracle's over the batch."""
    t_end = time.time() + BUDGET
    master = random.Random(int(os.environ.get("RXG_SOAK_SEED", "2027")))
    cases, t_print = 0, time.time()
    eng = rxg.Engine(device=0, max_batch=1 << 12, max_bytes=16 << 20)
    try:
        while time.time() < t_end:
            seed = master.randrange(1 << 30)
            rng = random.Random(seed)
            rows, frames = pktgen.parity_set(seed=seed, n=rng.choice([64, 300, 1000]), nflows=rng.choice([3, 50, 400]))
            tcb, live = pktgen.table_arrays(rows)
            kind = rng.choice([rxg.REC8, rxg.REC16, rxg.REC48])
            blocks = rng.choice([1, 3, 8])
            flags = rng.choice([0, rxg.SRV_HOST_STAGING, rxg.SRV_HOST_MAILBOX])
            arena, off, lens = pktgen.pack_arena(frames)
            exp, ecnt = oracle.rx_batch(arena, off, lens, tcb, live)
            exp = exp if kind == rxg.REC48 else exp["c"] if kind == rxg.REC16 else rxg.rec8_pack(exp["c"])
            eng.tcb_load(tcb, live)
            eng.counters_reset()
            eng.server_start(kind, blocks=blocks, max_frames=512, flags=flags)
            try:
                i, got = 0, []
                while i < len(frames):
                    k = min(len(frames) - i, rng.choice([1, 2, 7, 8, 31, 32, 33, 63, 64, 65, 100, 128, 129, 300]))
                    got.append(eng.rx_burst(frames[i:i + k], kind))
                    i += k
            finally:
                eng.server_stop()
            got = np.concatenate(got)
            assert got.tobytes() == exp.tobytes(), f"seed {seed} kind {kind} blocks {blocks} flags {flags}"
            assert eng.counters().tolist() == ecnt.tolist(), f"seed {seed}: counters differ"
            cases += 1
            if time.time() - t_print > 20:
                print(f"served soak: {cases} batches", flush=True)
                t_print = time.time()
    finally:
        eng.close()
    print(f"served soak: {cases} batches bit-exact")
    assert cases > 0


@pytest.mark.skipif(BUDGET <= 0, reason="opt-in soak: set RXG_SOAK=<seconds>")
def test_soak_fused_hand_off():
    """The burst with its payload hand-off in one pass (rxg_rx_burst_payload_dev, DESIGN.md
    §5.F) over random parity batches and grids: the copy form (payload lines into a sentinel
    arena) and the by-reference form (messages staged in the record ring, flushing mid-stream
    on small grids), every record kind -- records, counters, messages and payload bytes
    bit-exact with the oracle, and no line outside a payload written."""
    from oracle import payload as opl
    t_end = time.time() + BUDGET
    master = random.Random(int(os.environ.get("RXG_SOAK_SEED", "2028")))
    engines, cases, t_print = {}, 0, time.time()
    try:
        while time.time() < t_end:
            seed = master.randrange(1 << 30)
            rng = random.Random(seed)
            n = rng.choice([1, 31, 64, 65, 200, 1000, 4096, 9000])
            rows, frames = pktgen.parity_set(seed=seed, n=n, nflows=rng.choice([3, 50, 400]))
            for _ in range(rng.randrange(0, 4)):  # runs of small frames of a few flows
                a = rng.randrange(0, n)
                for i in range(a, min(n, a + rng.randrange(64, 700))):
                    frames[i] = pktgen.frame(src_ip=0x0A000001 + (i % 3), sport=1024 + (i % 3), dport=80,
                                             payload=bytes(rng.randrange(0, 11)))
            kind = rng.choice([rxg.REC8, rxg.REC16, rxg.REC48])
            blocks = rng.choice([0, 1, 2, 3, 5, 13, 40])  # 0: the product grid
            by_ref = rng.random() < 0.5
            if blocks not in engines:
                engines[blocks] = rxg.Engine(device=0, max_batch=1 << 14, max_bytes=32 << 20, max_blocks=blocks)
            eng = engines[blocks]
            tcb, live = pktgen.table_arrays(rows)
            eng.tcb_load(tcb, live)
            eng.counters_reset()
            recs, pay, msgs, (arena, off, lens) = eng.rx_burst_payload(frames, kind, arena_fill=0xA5,
                                                                       by_reference=by_ref)
            exp, ecnt = oracle.rx_batch(arena, off, lens, tcb, live)
            want = exp if kind == rxg.REC48 else exp["c"] if kind == rxg.REC16 else rxg.rec8_pack(exp["c"])
            what = f"seed {seed} n {n} kind {kind} blocks {blocks} by_ref {by_ref}"
            assert recs.tobytes() == want.tobytes(), what + ": records differ"
            assert eng.counters().tolist() == ecnt.tolist(), what + ": counters differ"
            e_msgs, pays = opl.slots(frames, exp["c"], off)
            for name in ("arena_off", "len", "flags"):
                assert np.array_equal(msgs[name], e_msgs[name]), what + f": msgs.{name} differ"
            mask = np.zeros(len(pay), dtype=bool)
            for i, p in enumerate(pays):
                if p is not None:
                    o = int(msgs[i]["arena_off"])
                    assert pay[o:o + len(p)].tobytes() == p, what + f": frame {i} payload differs"
                    mask[o // 64 * 64:(o + len(p) + 63) // 64 * 64] = True
            if not by_ref:
                assert (pay[~mask] == 0xA5).all(), what + ": a line holding no payload was written"
            cases += 1
            if time.time() - t_print > 20:
                print(f"fused soak: {cases} batches", flush=True)
                t_print = time.time()
    finally:
        for e in engines.values():
            e.close()
    print(f"fused soak: {cases} batches bit-exact")
    assert cases > 0
