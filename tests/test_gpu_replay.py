"""GPU: rxg_rx_burst + rxg_rx_replay equals the reference's sequential ether_in loop when the
state handlers change the TCB table inside a burst.

The handlers below mimic the kinds of writes tcp_states.c makes — tcp_listen allocates a
child TCB carrying the SYN's tuple (tcp_states.c:150-207), tcp_syn_rcv moves it to
ESTABLISHED, a FIN closes a flow and tcp_closed removes its slot (:209-219) — and mirror
each write with rxg_tcb_*.  The expected result is the oracle run ONE packet at a time
against the table as it stands when that packet is reached."""
import ctypes as C
import random

import numpy as np
import pytest

import oracle
import pktgen
import rxg

pytestmark = pytest.mark.gpu
LISTENING, SYN_RECV, ESTABLISHED, CLOSED = 1, 3, 4, 0
COUNTER_ROWS = 65  # rxg.h RXG_COUNTER_ROWS: 64 kernel replicas + the replay's corrections


class Model:
    """Table rows + the handler logic, applied identically to the python rows and rxg."""

    def __init__(self, rows, eng=None):
        self.rows = list(rows)
        self.eng = eng

    def _upsert(self, idx, row):
        while len(self.rows) <= idx:
            self.rows.append(None)
        self.rows[idx] = row
        if self.eng:
            self.eng.tcb_upsert(idx, row[0], row[1], row[2] & 0xFFFFFFFF, row[3] & 0xFFFFFFFF, row[4])

    def handle(self, idx, state, frame):
        flags = frame[47]
        sport = (frame[34] << 8) | frame[35]
        src = int.from_bytes(frame[26:30], "big")
        if state == LISTENING:          # tcp_listen: child at Ntcb with the SYN's tuple
            lst = self.rows[idx]
            self._upsert(len(self.rows), (lst[0], sport, lst[2], src, SYN_RECV))
        elif state == SYN_RECV:         # tcp_syn_rcv -> ESTABLISHED
            r = self.rows[idx]
            self.rows[idx] = r[:4] + (ESTABLISHED,)
            if self.eng:
                self.eng.tcb_set_state(idx, ESTABLISHED)
        elif state == ESTABLISHED and flags & 1:   # FIN: close
            r = self.rows[idx]
            self.rows[idx] = r[:4] + (CLOSED,)
            if self.eng:
                self.eng.tcb_set_state(idx, CLOSED)
        elif state == CLOSED:           # tcp_closed: remove_tcb
            self.rows[idx] = None
            if self.eng:
                self.eng.tcb_remove(idx)


def scenario(seed, nflows=40, n=1500, corrupt=0.0, closed=0.0):
    """Flows, listeners, unknown clients; `corrupt`: share of frames with one payload or
    header byte flipped after the checksums were filled (a bad TCP checksum); `closed`:
    share of client frames sent to a port nobody listens on (findtcb NULL, tcp_in.c:47)."""
    rng = random.Random(seed)
    dst = pktgen.ip4(192, 168, 78, 2)
    rows = [(80, 0, pktgen.raw_of_host(dst), 0, LISTENING)]
    flows = []
    for f in range(nflows):
        src = pktgen.ip4(10, 1, f >> 8, f & 255)
        rows.append((80, 2000 + f, pktgen.raw_of_host(dst), src, ESTABLISHED))
        flows.append((src, 2000 + f))
    rows.append((8080, 0, pktgen.raw_of_host(dst), 0, LISTENING))
    clients = [(pktgen.ip4(172, 16, 0, c), 40000 + c) for c in range(60)]
    frames = []
    for _ in range(n):
        k = rng.random()
        if k < 0.35:
            src, sport = rng.choice(flows)
            fl = 0x11 if rng.random() < 0.05 else 0x10
        else:
            src, sport = rng.choice(clients)
            fl = rng.choice([0x02, 0x10, 0x10, 0x18, 0x11])
        dport = 8080 if rng.random() < 0.1 else 80
        if closed and k >= 0.35 and rng.random() < closed:
            dport = 9999
        f = pktgen.frame(src_ip=src, dst_ip=dst, sport=sport, dport=dport, flags=fl,
                         seq=rng.getrandbits(32), ack=rng.getrandbits(32),
                         payload=rng.randbytes(rng.randrange(0, 200)))
        if corrupt and rng.random() < corrupt:
            b = bytearray(f)
            b[rng.randrange(38, len(b))] ^= 0x5A   # seq/ack/flags/payload: TCP checksum only
            f = bytes(b)
        frames.append(f)
    return rows, frames


def sequential_reference(rows, frames, verify=False, globals_out=None):
    """The reference loop: classify packet i against the table as it is NOW, then run its
    handler.  Returns per-packet (verdict, tcb_idx, state) and the summed counters.
    verify: tcp_in.c:37-40 compiled in -- a TCP segment with a bad checksum is freed before
    findtcb (verdict reported as V_DROP_NONTCP, "freed").  globals_out (dict) receives the
    reference's rx globals tcpnopcb (tcp_in.c:48) and tcpchecksumerror (:39)."""
    m = Model(rows)
    out, cnt = [], np.zeros(16, dtype=np.uint64)
    nopcb = cksumerr = 0
    for f in frames:
        arena, off, lens = pktgen.pack_arena([f])
        tcb, live = pktgen.table_arrays(m.rows)
        rec, c = oracle.rx_batch(arena, off, lens, tcb, live)
        cnt += c
        r = rec[0]["c"]
        v = int(r["verdict"])
        if verify and v in (rxg.V_DISPATCH, rxg.V_RST_NOPCB, rxg.V_RST_LISTEN_NONSYN) \
                and not (r["flags"] & rxg.F_TCP_OK):
            cksumerr += 1
            out.append((rxg.V_DROP_NONTCP, -1, rxg.STATE_NONE))
            continue
        nopcb += v == rxg.V_RST_NOPCB
        out.append((v, int(r["tcb_idx"]), int(r["state"])))
        if r["verdict"] == rxg.V_DISPATCH:
            m.handle(int(r["tcb_idx"]), int(r["state"]), f)
    if globals_out is not None:
        globals_out.update(tcpnopcb=nopcb, tcpchecksumerror=cksumerr)
    return out, cnt, m.rows


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_replay_sequential_equivalence(replay_engine, seed):
    run_replay_equivalence(replay_engine, seed)


def run_replay_equivalence(engine, seed, burst=None, check_counters=None):
    """burst(engine, frames) -> REC16 records: the burst form under test (default rxg_rx_burst).
    check_counters(engine, expected, rows, frames): in place of the counters read."""
    rows, frames = scenario(seed)
    exp, ecnt, erows = sequential_reference(rows, frames)
    tcb, live = pktgen.table_arrays(rows)
    engine.tcb_load(tcb, live)
    engine.tcb_sync()
    engine.counters_reset()
    recs = burst(engine, frames) if burst else engine.rx_burst(frames, rxg.REC16)
    model = Model(rows, engine)
    bufs = [C.create_string_buffer(f, max(len(f), 64)) for f in frames]
    addr = {C.addressof(b): i for i, b in enumerate(bufs)}
    got = [None] * len(frames)

    def free_mbuf(u, m):
        i = addr[m]
        if got[i] is None:
            got[i] = ("free",)
    def rst(u, ip, tcp):
        got[addr[ip - 14]] = ("rst",)
    def tcpswitch(u, idx, st, tcp, ip, m):
        i = addr[m]
        got[i] = ("switch", idx, st)
        model.handle(idx, st, frames[i])
        return 0

    ops = rxg.HandoffOps(None, rxg.HANDOFF_FREE(free_mbuf), rxg.HANDOFF_ARP_IN(), rxg.HANDOFF_GET_MAC(),
                         rxg.HANDOFF_ADD_MAC(), rxg.HANDOFF_SEND_RESET(rst), rxg.HANDOFF_ON_SEGMENT(),
                         rxg.HANDOFF_TCPSWITCH(tcpswitch))
    ptrs = (C.c_void_p * len(bufs))(*[C.addressof(b) for b in bufs])
    lib = rxg.load_library()
    rc = lib.rxg_rx_replay(engine.ctx, C.byref(ops), ptrs, ptrs, recs.ctypes.data, len(bufs), 16)
    assert rc == 0, lib.rxg_last_error()
    for i, (v, idx, st) in enumerate(exp):
        if v == rxg.V_DISPATCH:
            assert got[i] == ("switch", idx, st), (i, got[i], exp[i])
        elif v in (rxg.V_RST_NOPCB, rxg.V_RST_LISTEN_NONSYN):
            assert got[i] == ("rst",), (i, got[i], exp[i])
    assert model.rows == erows
    if check_counters:
        check_counters(engine, ecnt, erows, frames)
    else:
        assert engine.counters().tolist() == ecnt.tolist()
    # the burst alone (snapshot semantics) would have differed: the scenario bites
    snap = [(int(r["verdict"]), int(r["tcb_idx"]), int(r["state"])) for r in recs]
    assert snap != exp


def test_arp_learn_flag_and_replay(engine):
    """ip.c:30-32 with the ARP mirror: the burst flags TCP packets from unknown sources and
    the replay calls add_mac once per new address, in first-seen order, never get_mac."""
    rng = random.Random(9)
    known = [pktgen.ip4(10, 0, 0, k) for k in range(20)]
    unknown = [pktgen.ip4(10, 9, 0, k) for k in range(30)]
    frames = []
    for _ in range(800):
        k = rng.random()
        if k < 0.1:   # ARP and non-TCP frames never learn
            frames.append(pktgen.frame(proto=17, src_ip=rng.choice(unknown)))
            continue
        src = rng.choice(known if k < 0.5 else unknown)
        frames.append(pktgen.frame(src_ip=src, sport=rng.randrange(65536), flags=0x10))
    tcb, live = pktgen.table_arrays([(80, 0, pktgen.raw_of_host(pktgen.ip4(192, 168, 78, 2)), 0, 1)])
    engine.tcb_load(tcb, live)
    engine.arp_load(known)
    recs = engine.rx_burst(frames, rxg.REC16)
    # flag: TCP and source not in the mirror at burst time
    for f, r in zip(frames, recs):
        is_tcp = r["verdict"] in (0, 1, 2)
        src = int.from_bytes(f[26:30], "big")
        assert bool(r["flags"] & rxg.F_ARP_LEARN) == (is_tcp and src not in known)
    # reference order of add_mac: first TCP sighting of each unknown source
    exp, seen = [], set(known)
    for f, r in zip(frames, recs):
        if r["verdict"] in (0, 1, 2):
            src = int.from_bytes(f[26:30], "big")
            if src not in seen:
                seen.add(src)
                exp.append(src)
    calls = []

    def add_mac(u, ip, mac):
        calls.append(ip)
        engine.arp_learned(ip)   # the integration's add_mac hook
        return 1

    def get_mac(u, ip, out):
        raise AssertionError("get_mac walked while the ARP mirror is enabled")

    bufs = [C.create_string_buffer(f, max(len(f), 64)) for f in frames]
    ops = rxg.HandoffOps(None, rxg.HANDOFF_FREE(), rxg.HANDOFF_ARP_IN(), rxg.HANDOFF_GET_MAC(get_mac),
                         rxg.HANDOFF_ADD_MAC(add_mac), rxg.HANDOFF_SEND_RESET(), rxg.HANDOFF_ON_SEGMENT(),
                         rxg.HANDOFF_TCPSWITCH())
    ptrs = (C.c_void_p * len(bufs))(*[C.addressof(b) for b in bufs])
    lib = rxg.load_library()
    assert lib.rxg_rx_replay(engine.ctx, C.byref(ops), ptrs, ptrs, recs.ctypes.data, len(bufs), 16) == 0
    assert calls == exp
    assert engine.arp_count() == len(known) + len(exp)
    # a TCB write beside the learned addresses: the next burst takes both mirrors' patches
    # (one list the burst itself carries on a large-BAR box)
    dst_raw = pktgen.raw_of_host(pktgen.ip4(192, 168, 78, 2))
    engine.tcb_upsert(1, 80, 5555, dst_raw, unknown[0], 4)
    probe = [pktgen.frame(src_ip=unknown[0], sport=5555, flags=0x10)] + frames
    recs_b = engine.rx_burst(probe, rxg.REC16)
    assert int(recs_b[0]["verdict"]) == rxg.V_DISPATCH and int(recs_b[0]["tcb_idx"]) == 1
    assert not (recs_b["flags"] & rxg.F_ARP_LEARN).any()
    engine.tcb_remove(1)
    # a second burst of the same frames learns nothing new
    recs2 = engine.rx_burst(frames, rxg.REC16)
    assert not (recs2["flags"] & rxg.F_ARP_LEARN).any()
    engine.arp_disable()
    recs3 = engine.rx_burst(frames, rxg.REC16)
    assert not (recs3["flags"] & rxg.F_ARP_LEARN).any()


def test_replay_refused_after_a_failed_burst(engine):
    """A burst that fails after it started (staging full) leaves nothing to replay: the
    replay of the same n is refused instead of replaying the previous burst's records."""
    n = 45000
    small = [pktgen.frame(sport=1000 + i % 50) for i in range(n)]
    big = [pktgen.frame(sport=1000, payload=bytes(1446))] * n   # 67.5 MB > staging
    recs = engine.rx_burst(small, rxg.REC16)
    lib = rxg.load_library()
    ops = rxg.HandoffOps()
    bufs = [C.create_string_buffer(f, 64) for f in small[:1]] * n
    ptrs = (C.c_void_p * n)(*[C.addressof(b) for b in bufs])
    assert lib.rxg_rx_replay(engine.ctx, C.byref(ops), ptrs, ptrs, recs.ctypes.data, n, 16) == 0
    with pytest.raises(rxg.RxgError, match="staging arena"):
        engine.rx_burst(big, rxg.REC16)
    assert lib.rxg_rx_replay(engine.ctx, C.byref(ops), ptrs, ptrs, recs.ctypes.data, n, 16) == -22
    assert b"failed" in lib.rxg_last_error()


def _arp_hash(ip):
    """rxg_common.h arp_hash (murmur3 finaliser), to build bucket clusters on purpose."""
    M = 0xFFFFFFFF
    h = (ip ^ 0x41525000) & M
    h ^= h >> 16
    h = (h * 0x85EBCA6B) & M
    h ^= h >> 13
    h = (h * 0xC2B2AE35) & M
    return h ^ (h >> 16)


def test_arp_bucket_clusters_and_zero(engine):
    """The ARP mirror's bucketed probe: addresses whose first bucket is full (clusters over
    several buckets, found and not found), 0.0.0.0 (a launch flag, not a key), additions by
    patch (rxg_arp_learned) and by rebuild, over small-frame and streaming slices."""
    rng = random.Random(31)
    def nb_for(n):
        nb = 4
        while nb * 4 < 2 * n:
            nb <<= 1
        return nb
    # 40 known: 14 with first bucket 5 (fill buckets 5..8), the rest anywhere
    mask = nb_for(40) - 1
    pool = [pktgen.ip4(10, 77, rng.randrange(256), rng.randrange(1, 256)) for _ in range(20000)]
    pool = list(dict.fromkeys(pool))
    clus = [ip for ip in pool if _arp_hash(ip) & mask == 5]
    assert len(clus) >= 30
    known = clus[:14] + [ip for ip in pool if _arp_hash(ip) & mask != 5][:26]
    unknown = clus[14:24] + [ip for ip in pool if ip not in known][100:120] + [0]
    srcs = known + unknown
    frames = [pktgen.frame(src_ip=rng.choice(srcs), sport=rng.randrange(1024, 65536), flags=0x10,
                           payload=bytes(rng.choice([0, 0, 0, 10, 600, 1400]))) for _ in range(3000)]
    tcb, live = pktgen.table_arrays([(80, 0, pktgen.raw_of_host(pktgen.ip4(192, 168, 78, 2)), 0, 1)])
    engine.tcb_load(tcb, live)
    engine.arp_load(known)

    def check(members):
        for kind in (rxg.REC16, rxg.REC8):
            recs = engine.rx_burst(frames, kind)
            if kind == rxg.REC8:
                fl = (recs["w1"] >> 8) & 0x3F
            else:
                fl = recs["flags"]
            got = (fl & rxg.F_ARP_LEARN) != 0
            exp = np.array([int.from_bytes(f[26:30], "big") not in members for f in frames])
            assert (got == exp).all(), (kind, np.flatnonzero(got != exp)[:8])

    check(set(known))
    for ip in clus[14:24]:              # patches into the cluster (no rebuild: load <= 1/2)
        engine.arp_learned(ip)
    check(set(known) | set(clus[14:24]))
    engine.arp_learned(0)
    check(set(known) | set(clus[14:24]) | {0})
    for ip in pool[:200]:               # past load 1/2: rebuilt at a larger size
        engine.arp_learned(ip)
    check(set(known) | set(clus[14:24]) | {0} | set(pool[:200]))
    engine.arp_disable()


@pytest.mark.parametrize("path", ["dev_pointer", "reset", "next_burst"])
def test_replay_corrections_reach_the_counter_block(replay_engine, path):
    """The replay's counter corrections wait on the host for the context's next mirror patch
    launch (csrc/rxg_replay.cpp, rxg_host.cpp flush_delta): read through rxg_counters_dev
    after rxg_sync they are in the device block; a reset before the next burst zeroes them
    with the rest; the next burst's patch launch carries them (its own counts added)."""
    lib = rxg.load_library()

    def check(engine, ecnt, rows, frames):
        if path == "dev_pointer":
            ptr = lib.rxg_counters_dev(engine.ctx)
            block = np.zeros(COUNTER_ROWS * 16, dtype=np.uint64)
            assert lib.rxg_memcpy_d2h(engine.ctx, block.ctypes.data, ptr, block.nbytes, None) == 0
            engine.sync()
            assert block.reshape(COUNTER_ROWS, 16).sum(axis=0).tolist() == ecnt.tolist()
        elif path == "reset":
            engine.counters_reset()
            assert engine.counters().tolist() == [0] * 16
        else:
            arena, off, lens = pktgen.pack_arena(frames)
            tcb, live = pktgen.table_arrays(rows)
            _, c2 = oracle.rx_batch(arena, off, lens, tcb, live)  # the next burst, against the new table
            engine.rx_burst(frames, rxg.REC16)
            assert engine.counters().tolist() == (ecnt + c2).tolist()

    run_replay_equivalence(replay_engine, 4, check_counters=check)
