"""CPU tests of the oracle (the checker) — pinned against the KATs and cross-checked
against an independent pure-Python restatement of the reference rx path."""
import json
import os
import random
import struct

import numpy as np
import pytest

import oracle
import pktgen

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def _kat():
    with open(os.path.join(GOLD, "kat.json")) as fh:
        return json.load(fh)


@pytest.mark.parametrize("case", _kat()["checksum"], ids=lambda c: c["source"])
def test_checksum_kat(case):
    data = bytes.fromhex(case["hex"])
    assert oracle.calculate_checksum(data) == case["expect"]
    assert pktgen.py_checksum(data) == case["expect"]


def test_checksum_random_vs_python():
    rng = random.Random(1)
    for _ in range(2000):
        d = rng.randbytes(rng.randrange(0, 3000))
        assert oracle.calculate_checksum(d) == pktgen.py_checksum(d)


# ------------------------------------------------------- pure-Python rx restatement ---
def py_rx(f: bytes, rows):
    """etherin.c:12-37 -> ip.c:19-42 -> tcp_in.c:32-84 -> tcp_tcb.c:127-173, one frame."""
    g = (f + b"\0" * 54)[:54]
    et, tl = struct.unpack(">H", g[12:14])[0], struct.unpack(">H", g[16:18])[0]
    vihl, proto, doff, fl = g[14], g[23], g[46], g[47]
    sport, dport = struct.unpack(">HH", g[34:38])
    src = struct.unpack(">I", g[26:30])[0]
    dst_raw = struct.unpack("<I", g[30:34])[0]
    r = dict(ether_type=et, sport=sport, dport=dport, l4_proto=proto, version_ihl=vihl,
             seq=struct.unpack(">I", g[38:42])[0], ack=struct.unpack(">I", g[42:46])[0],
             src_ip=src, dst_ip_raw=dst_raw, data_off=doff, tcp_flags=fl,
             datalen=tl - (vihl & 15) * 4 - (doff >> 4) * 4, tcb_idx=-1, state=0xFF,
             ip_cksum=0, tcp_cksum=0, flags=16 if len(f) < 54 else 0)
    if et == 0x0806:
        r["verdict"] = 4
        return r
    if et != 0x0800:
        r["verdict"] = 5
        return r
    r["ip_cksum"] = pktgen.ip_checksum_of(f)
    r["flags"] |= 1 if r["ip_cksum"] == 0 else 0
    if proto != 6:
        r["verdict"] = 3
        return r
    r["tcp_cksum"] = pktgen.tcp_checksum_of(f)
    r["flags"] |= 2 if r["tcp_cksum"] == 0 else 0
    idx = -1
    for i, t in enumerate(rows):  # pass 1
        if t is not None and t[0] == dport and t[1] == sport and (t[2] & 0xFFFFFFFF) == dst_raw \
                and (t[3] & 0xFFFFFFFF) == src:
            idx = i
            break
    if idx < 0:  # pass 2
        for i, t in enumerate(rows):
            if t is None:
                r["flags"] |= 8
                continue
            if t[4] == 1 and t[0] == dport:
                idx = i
                r["flags"] |= 4
                break
    r["tcb_idx"] = idx
    if idx < 0:
        r["verdict"] = 1
        return r
    r["state"] = rows[idx][4]
    r["verdict"] = 2 if (r["state"] == 1 and not (fl & 2)) else 0
    return r


def _cmp(rec, ref):
    got = dict(ether_type=rec["ether_type"], sport=rec["sport"], dport=rec["dport"],
               l4_proto=rec["l4_proto"], version_ihl=rec["version_ihl"], seq=rec["seq"],
               ack=rec["ack"], src_ip=rec["src_ip"], dst_ip_raw=rec["dst_ip_raw"],
               data_off=rec["data_off"], tcp_flags=rec["c"]["tcp_flags"],
               datalen=rec["c"]["datalen"], tcb_idx=rec["c"]["tcb_idx"], state=rec["c"]["state"],
               ip_cksum=rec["c"]["ip_cksum"], tcp_cksum=rec["c"]["tcp_cksum"],
               flags=rec["c"]["flags"], verdict=rec["c"]["verdict"])
    got = {k: int(v) for k, v in got.items()}
    assert got == ref


def test_oracle_vs_python_restatement():
    rows, frames = pktgen.parity_set(seed=7, n=1500)
    arena, off, lens = pktgen.pack_arena(frames)
    tcb, live = pktgen.table_arrays(rows)
    rec, _ = oracle.rx_batch(arena, off, lens, tcb, live)
    for i, f in enumerate(frames):
        _cmp(rec[i], py_rx(f, rows))
        assert bytes(rec[i]["src_mac"]) == (f + b"\0" * 12)[6:12]


def test_faithful_mode_same_records():
    rows, frames = pktgen.parity_set(seed=8, n=400)
    arena, off, lens = pktgen.pack_arena(frames)
    tcb, live = pktgen.table_arrays(rows)
    a, ca = oracle.rx_batch(arena, off, lens, tcb, live)
    oracle.arp_reset()
    b, cb = oracle.rx_batch(arena, off, lens, tcb, live, faithful=True)
    c, cc = oracle.rx_batch(arena, off, lens, tcb, live, faithful=True, opt="O0")
    assert a.tobytes() == b.tobytes() == c.tobytes()
    assert np.array_equal(ca, cb) and np.array_equal(ca, cc)
    # ARP list learned one entry per distinct TCP source (ip.c:30-32)
    tcp_src = {int(r["src_ip"]) for r in a if r["ether_type"] == 0x0800 and r["l4_proto"] == 6}
    assert oracle.lib().orc_arp_count() == len(tcp_src)
    oracle.arp_reset()


def test_counters_definition():
    rows, frames = pktgen.parity_set(seed=9, n=600)
    arena, off, lens = pktgen.pack_arena(frames)
    tcb, live = pktgen.table_arrays(rows)
    rec, cnt = oracle.rx_batch(arena, off, lens, tcb, live)
    v = rec["c"]["verdict"]
    assert cnt[0] == len(frames) and cnt[1] == int(lens.astype(np.uint64).sum())
    assert cnt[2] == int((rec["ether_type"] == 0x0800).sum())
    assert cnt[3] == int((v == 4).sum()) and cnt[4] == int((v == 5).sum())
    assert cnt[11] == int((v == 1).sum()) and cnt[12] == int((v == 2).sum())
    assert cnt[13] == int((v == 0).sum())
    assert cnt[5] == cnt[9] + cnt[10] + cnt[11]


def test_tx_then_rx_roundtrip():
    """ip_out-generated checksums verify to 0x0000 (SURVEY.md §4 round-trip property)."""
    rng = random.Random(3)
    frames = []
    for _ in range(300):
        f = pktgen.frame(src_ip=rng.getrandbits(32), sport=rng.randrange(65536),
                         payload=rng.randbytes(rng.randrange(0, 1600)), valid_ip=False,
                         valid_tcp=False)
        frames.append(f)
    arena, off, lens = pktgen.pack_arena(frames)
    out = oracle.tx_batch(arena, off, lens)
    rec, _ = oracle.rx_batch(out, off, lens, np.zeros(0, dtype=oracle.TCB_DTYPE))
    assert (rec["c"]["ip_cksum"] == 0).all() and (rec["c"]["tcp_cksum"] == 0).all()
    # and equals the Python builder's own valid checksums
    for i, f in enumerate(frames):
        o = int(off[i]) * 64
        g = bytes(out[o:o + len(f)])
        assert pktgen.ip_checksum_of(g) == 0 and pktgen.tcp_checksum_of(g) == 0


def test_classify_kat():
    kat = _kat()["classify"]
    dst = pktgen.ip4(192, 168, 78, 2)
    rows = [(80, 0, pktgen.raw_of_host(dst), 0, 1),
            (80, 1024, pktgen.raw_of_host(dst), pktgen.ip4(10, 0, 0, 1), 4)]
    tcb, live = pktgen.table_arrays(rows)
    frames = []
    for c in kat:
        a, b, cc, d = (int(x) for x in c["src"].split("."))
        frames.append(pktgen.frame(src_ip=pktgen.ip4(a, b, cc, d), dst_ip=dst, sport=c["sport"],
                                   dport=c["dport"], flags=c["flags"]))
    arena, off, lens = pktgen.pack_arena(frames)
    rec, _ = oracle.rx_batch(arena, off, lens, tcb, live)
    for r, c in zip(rec, kat):
        assert int(r["c"]["verdict"]) == c["expect_verdict"], c["case"]
        assert int(r["c"]["tcb_idx"]) == c["expect_tcb"], c["case"]


def test_golden_rx_regression():
    g = np.load(os.path.join(GOLD, "rx_golden.npz"))
    rec, cnt = oracle.rx_batch(g["arena"], g["off64"], g["len"], g["tcb"], g["live"])
    assert rec.tobytes() == g["records"].tobytes()
    assert np.array_equal(cnt, g["counters"])
    # the set covers every verdict and every record flag
    assert set(np.unique(rec["c"]["verdict"]).tolist()) == {0, 1, 2, 3, 4, 5}
    for bit in (1, 2, 4, 8, 16):
        assert (rec["c"]["flags"] & bit).any(), bit


def test_golden_tx_regression():
    g = np.load(os.path.join(GOLD, "rx_golden.npz"))
    t = np.load(os.path.join(GOLD, "tx_golden.npz"))
    arena, off, lens = g["arena"].copy(), g["off64"], g["len"]
    pos = (off.astype(np.int64) * 64)[:, None] + np.array([24, 25, 50, 51])[None, :]
    inside = pos < (off.astype(np.int64) * 64 + lens.astype(np.int64))[:, None]
    arena[pos[inside]] = 0
    out = oracle.tx_batch(arena, off, lens)
    assert np.array_equal(out[pos], t["cksum_bytes"])


def test_shipped_mode_classifies_as_faithful():
    """orc_rx_batch_shipped (timing only: the reference as shipped, tcp_in.c:37's verify
    compiled out) gives the faithful path's classification, with no checksum fields."""
    rows, frames = pktgen.parity_set(seed=7, n=800)
    arena, off, lens = pktgen.pack_arena(frames)
    tcb, live = pktgen.table_arrays(rows)
    oracle.arp_reset()
    a, ca = oracle.rx_batch(arena, off, lens, tcb, live, faithful=True)
    oracle.arp_reset()
    b, cb = oracle.rx_batch(arena, off, lens, tcb, live, faithful=True, shipped=True)
    oracle.arp_reset()
    for k in ("tcb_idx", "verdict", "state", "datalen", "tcp_flags"):
        assert (a["c"][k] == b["c"][k]).all(), k
    assert not b["c"]["ip_cksum"].any() and not b["c"]["tcp_cksum"].any()
    ok = 0x01 | 0x02  # RXG_F_IP_OK | RXG_F_TCP_OK
    assert ((a["c"]["flags"] & np.uint8(0xFF ^ ok)) == b["c"]["flags"]).all()
