"""GPU parity: rxg's HIP path (through the C ABI) vs the oracle, bit-exact."""
import os
import random

import numpy as np
import pytest

import oracle
import pktgen
import rxg

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")

REC_FIELDS = ["ether_type", "sport", "dport", "l4_proto", "version_ihl", "seq", "ack", "src_ip",
              "dst_ip_raw", "data_off", "src_mac", "reserved"]
C_FIELDS = ["tcb_idx", "ip_cksum", "tcp_cksum", "verdict", "state", "tcp_flags", "flags", "datalen"]


def assert_records_equal(got, exp, frames=None):
    if got.tobytes() == exp.tobytes():
        return
    for name in C_FIELDS:
        bad = np.nonzero(got["c"][name] != exp["c"][name])[0]
        if len(bad):
            i = int(bad[0])
            extra = f" len={len(frames[i])}" if frames is not None else ""
            raise AssertionError(f"c.{name} differs at {len(bad)} frames, first {i}{extra}: "
                                 f"got {got['c'][name][i]} exp {exp['c'][name][i]}")
    for name in REC_FIELDS:
        g, e = got[name], exp[name]
        bad = np.nonzero((g != e).reshape(len(g), -1).any(axis=1))[0]
        if len(bad):
            i = int(bad[0])
            raise AssertionError(f"{name} differs at {len(bad)} frames, first {i}: "
                                 f"got {g[i]} exp {e[i]}")
    raise AssertionError("records differ")


def run_both(engine, rows, frames, rec_kind=rxg.REC48):
    arena, off, lens = pktgen.pack_arena(frames)
    tcb, live = pktgen.table_arrays(rows)
    engine.tcb_load(tcb, live)
    engine.counters_reset()
    got = engine.rx_arena(arena, off, lens, rec_kind)
    cnt = engine.counters()
    exp, ecnt = oracle.rx_batch(arena, off, lens, tcb, live)
    return got, cnt, exp, ecnt


def test_golden_fixture(engine):
    g = np.load(os.path.join(GOLD, "rx_golden.npz"))
    engine.tcb_load(g["tcb"], g["live"])
    engine.counters_reset()
    got = engine.rx_arena(g["arena"], g["off64"], g["len"], rxg.REC48)
    assert_records_equal(got, g["records"])
    assert np.array_equal(engine.counters(), g["counters"])


def test_golden_fixture_rec16(engine):
    g = np.load(os.path.join(GOLD, "rx_golden.npz"))
    engine.tcb_load(g["tcb"], g["live"])
    got = engine.rx_arena(g["arena"], g["off64"], g["len"], rxg.REC16)
    assert got.tobytes() == g["records"]["c"].tobytes()


@pytest.mark.parametrize("seed", [11, 12, 13])
def test_random_parity_sets(engine, seed):
    rows, frames = pktgen.parity_set(seed=seed, n=6000)
    got, cnt, exp, ecnt = run_both(engine, rows, frames)
    assert_records_equal(got, exp, frames)
    assert np.array_equal(cnt, ecnt)


def test_every_length_0_to_2100(engine):
    """Every data_len across all size classes, valid and corrupted frames."""
    rng = random.Random(5)
    rows, flows, _ = pktgen.parity_table(rng, 50)
    frames = []
    for L in range(0, 2101):
        src, sport, dport = rng.choice(flows)
        full = pktgen.frame(src_ip=src, sport=sport, dport=dport, payload=rng.randbytes(max(0, L - 54)))
        frames.append(full[:L])
        bad = bytearray(full[:L])
        if L > 60:
            bad[rng.randrange(54, L)] ^= 0xFF
        frames.append(bytes(bad))
    got, cnt, exp, ecnt = run_both(engine, rows, frames)
    assert_records_equal(got, exp, frames)
    assert np.array_equal(cnt, ecnt)


def test_jumbo_and_max_length(engine):
    rng = random.Random(6)
    rows, flows, _ = pktgen.parity_table(rng, 20)
    frames = []
    for L in [2049, 3000, 4096, 4097, 8191, 9000, 9018, 16384, 32768, 65535]:
        src, sport, dport = rng.choice(flows)
        f = pktgen.frame(src_ip=src, sport=sport, dport=dport, payload=rng.randbytes(L - 54),
                         total_length=(L - 14) & 0xFFFF)
        frames.append(f[:L])
        frames.append(pktgen.frame(src_ip=src, sport=sport, dport=dport,
                                   payload=rng.randbytes(min(L, 65481) - 54))[:L])
    got, cnt, exp, ecnt = run_both(engine, rows, frames)
    assert_records_equal(got, exp, frames)


def test_empty_batch_and_empty_table(engine):
    engine.tcb_load(np.zeros(0, dtype=rxg.TCB_DTYPE))
    got = engine.rx_arena(np.zeros(64, np.uint8), np.zeros(0, np.uint32), np.zeros(0, np.uint16))
    assert len(got) == 0
    rows, frames = [], [pktgen.frame(payload=b"x" * 100) for _ in range(100)]
    got, cnt, exp, ecnt = run_both(engine, rows, frames)
    assert_records_equal(got, exp)
    assert (got["c"]["verdict"] == rxg.V_RST_NOPCB).all()


def test_mirror_mutations(engine):
    """rxg_tcb_upsert/remove/set_state mirror the reference's tcbs[] writes."""
    rng = random.Random(21)
    rows, frames = pktgen.parity_set(seed=21, n=3000)
    tcb, live = pktgen.table_arrays(rows)
    engine.tcb_load(tcb, live)
    ops = [("remove", 0), ("state", 3, 1), ("remove", 5), ("upsert", len(rows) + 3, rows[7]),
           ("state", 2, 4), ("upsert", 0, (80, 0, rows[1][2], 0, 1))]
    for op in ops:
        if op[0] == "remove":
            rows[op[1]] = None
            engine.tcb_remove(op[1])
        elif op[0] == "state":
            if rows[op[1]] is not None:
                rows[op[1]] = rows[op[1]][:4] + (op[2],)
                engine.tcb_set_state(op[1], op[2])
        else:
            idx, r = op[1], op[2]
            while len(rows) <= idx:
                rows.append(None)
            rows[idx] = r
            engine.tcb_upsert(idx, r[0], r[1], r[2] & 0xFFFFFFFF, r[3] & 0xFFFFFFFF, r[4])
        assert engine.tcb_count() == len(rows)
        arena, off, lens = pktgen.pack_arena(frames)
        got = engine.rx_arena(arena, off, lens, rxg.REC48)
        t2, l2 = pktgen.table_arrays(rows)
        exp, _ = oracle.rx_batch(arena, off, lens, t2, l2)
        assert_records_equal(got, exp, frames)
    del rng


def test_large_table_collisions(engine):
    """20k TCBs (the reference's cap) + 200k beyond it, duplicates interleaved."""
    rng = random.Random(31)
    dst = pktgen.raw_of_host(pktgen.ip4(192, 168, 78, 2))
    n = 220_000
    rows = [(80, 0, dst, 0, 1)]
    for f in range(n):
        rows.append((80, 1024 + (f * 7919) % 64511, dst, (10 << 24) | (f * 2654435761 % (1 << 24)), 4))
    for k in range(0, n, 997):  # duplicates at higher indices never win
        rows.append(rows[1 + k])
    frames = []
    for _ in range(5000):
        r = rows[rng.randrange(len(rows))]
        frames.append(pktgen.frame(src_ip=r[3], sport=r[1], dport=r[0], flags=rng.choice([2, 16]),
                                   payload=rng.randbytes(rng.randrange(0, 100))))
    got, cnt, exp, ecnt = run_both(engine, rows, frames)
    assert_records_equal(got, exp, frames)
    assert np.array_equal(cnt, ecnt)


def test_host_burst_matches_device_burst(engine):
    rows, frames = pktgen.parity_set(seed=41, n=2000)
    tcb, live = pktgen.table_arrays(rows)
    engine.tcb_load(tcb, live)
    a = engine.rx_burst(frames, rxg.REC48)
    arena, off, lens = pktgen.pack_arena(frames)
    exp, _ = oracle.rx_batch(arena, off, lens, tcb, live)
    assert_records_equal(a, exp, frames)


def test_large_host_bursts_use_the_packing_pool(engine):
    """Host bursts over 4 MiB are packed by several threads (rxg_rx_burst's pool, kept for
    the context's life): two such bursts in a row, records equal to the device path's."""
    rng = np.random.default_rng(43)
    rows = [(80, 0, pktgen.raw_of_host(pktgen.ip4(192, 168, 78, 2)), 0, 1)]
    tcb, live = pktgen.table_arrays(rows)
    engine.tcb_load(tcb, live)
    for k in range(2):
        frames = [pktgen.frame(sport=1000 + i % 5000, payload=rng.bytes(int(rng.integers(0, 1400))))
                  for i in range(24000)]
        got = engine.rx_burst(frames, rxg.REC8)
        arena, off, lens = pktgen.pack_arena(frames)
        assert arena.size > (12 << 20)  # at least three packing threads
        assert got.tobytes() == engine.rx_arena(arena, off, lens, rxg.REC8).tobytes()


def test_tx_generate_golden(engine):
    g = np.load(os.path.join(GOLD, "rx_golden.npz"))
    t = np.load(os.path.join(GOLD, "tx_golden.npz"))
    arena, off, lens = g["arena"].copy(), g["off64"], g["len"]
    pos = (off.astype(np.int64) * 64)[:, None] + np.array([24, 25, 50, 51])[None, :]
    inside = pos < (off.astype(np.int64) * 64 + lens.astype(np.int64))[:, None]
    arena[pos[inside]] = 0
    out = engine.tx_arena(arena, off, lens)
    assert np.array_equal(out[pos], t["cksum_bytes"])
    assert np.array_equal(np.delete(out, pos.ravel()), np.delete(arena, pos.ravel()))


def test_tx_generate_random(engine):
    rows, frames = pktgen.parity_set(seed=51, n=5000)
    arena, off, lens = pktgen.pack_arena(frames)
    got = engine.tx_arena(arena, off, lens)
    exp = oracle.tx_batch(arena, off, lens)
    assert np.array_equal(got, exp)


def test_replay_order_and_side_effects(engine):
    """rxg_rx_replay performs ether_in's side effects in packet order."""
    import ctypes as C
    rows, frames = pktgen.parity_set(seed=61, n=500)
    tcb, live = pktgen.table_arrays(rows)
    engine.tcb_load(tcb, live)
    rec = engine.rx_arena(*pktgen.pack_arena(frames), rxg.REC16)
    log = []
    bufs = [C.create_string_buffer(f, max(len(f), 64)) for f in frames]
    addr = {C.addressof(b): i for i, b in enumerate(bufs)}
    arp = {}

    def free_mbuf(u, m): log.append(("free", addr[m]))
    def arp_in(u, m): log.append(("arp_in", addr[m])); return 0
    def get_mac(u, ip, out): return 1 if ip in arp else 0
    def add_mac(u, ip, mac): arp[ip] = C.string_at(mac, 6); log.append(("add_mac", ip)); return 1
    def send_reset(u, ip, tcp): log.append(("rst", addr[ip - 14]))
    def on_seg(u, idx, seq, ack): log.append(("seg", idx, seq, ack))
    def tcpswitch(u, idx, st, tcp, ip, m): log.append(("switch", idx, st, addr[m])); return 0

    ops = rxg.HandoffOps(None, rxg.HANDOFF_FREE(free_mbuf), rxg.HANDOFF_ARP_IN(arp_in),
                         rxg.HANDOFF_GET_MAC(get_mac), rxg.HANDOFF_ADD_MAC(add_mac),
                         rxg.HANDOFF_SEND_RESET(send_reset), rxg.HANDOFF_ON_SEGMENT(on_seg),
                         rxg.HANDOFF_TCPSWITCH(tcpswitch))
    ptrs = (C.c_void_p * len(bufs))(*[C.addressof(b) for b in bufs])
    rc = rxg.load_library().rxg_rx_replay(engine.ctx, C.byref(ops), ptrs, ptrs,
                                           rec.ctypes.data, len(bufs), 16)
    assert rc == 0
    # expected log from the reference's control flow
    exp, arp2 = [], {}
    import struct
    for i, (f, r) in enumerate(zip(frames, rec)):
        v = int(r["verdict"])
        if v == rxg.V_ARP:
            exp += [("arp_in", i), ("free", i)]
        elif v in (rxg.V_DROP_L2, rxg.V_DROP_NONTCP):
            exp.append(("free", i))
        else:
            g = f + b"\0" * 64
            src = struct.unpack(">I", g[26:30])[0]
            if src not in arp2:
                arp2[src] = 1
                exp.append(("add_mac", src))
            if v in (rxg.V_RST_NOPCB, rxg.V_RST_LISTEN_NONSYN):
                exp += [("free", i), ("rst", i)]
            else:
                seq, ack = struct.unpack(">II", g[38:46])
                exp += [("seg", int(r["tcb_idx"]), seq, ack), ("switch", int(r["tcb_idx"]), int(r["state"]), i)]
    assert log == exp
