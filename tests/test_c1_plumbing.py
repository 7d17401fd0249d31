"""Config 1 (plumbing): socket_tester-style listener <-> scripted samplesocketclient peer,
one TCP flow, handshake -> data -> FIN.  The CPU test runs the reference rx path (the
oracle, one packet at a time) — no GPU; the GPU test runs the same exchange through rxg
(burst + in-order replay + tx checksum generate) and must produce the same bytes."""
import ctypes as C
import struct

import numpy as np
import pytest

import c1_stack as c1
import oracle
import pktgen

MESSAGES = [b"Hello World %d" % i for i in range(5)] + [bytes(range(256)) * 5]


def with_checksums(f: bytes) -> bytes:
    """The peer's own (Linux) stack fills both checksums."""
    g = bytearray(f)
    g[24:26] = b"\0\0"
    g[24:26] = struct.pack(">H", pktgen.ip_checksum_of(bytes(g)))
    g[50:52] = b"\0\0"
    g[50:52] = struct.pack(">H", pktgen.tcp_checksum_of(bytes(g)))
    return bytes(g)


def run_cpu(one_burst):
    """The reference rx loop: ether_in per packet against the table as it stands."""
    st = c1.Stack()
    for burst in c1.peer_script(MESSAGES, one_burst):
        for f in map(with_checksums, burst):
            arena, off, lens = pktgen.pack_arena([f])
            tcb, live = pktgen.table_arrays(st.rows)
            rec, _ = oracle.rx_batch(arena, off, lens, tcb, live)
            r = rec[0]["c"]
            assert r["ip_cksum"] == 0 and r["tcp_cksum"] == 0
            if r["verdict"] == 0:
                st.tcpswitch(int(r["tcb_idx"]), int(r["state"]), f, int(r["datalen"]))
            elif r["verdict"] in (1, 2):
                st.send_reset(f)
        # ip_out: the tx frames get their checksums
        if st.tx:
            arena, off, lens = pktgen.pack_arena(st.tx)
            out = oracle.tx_batch(arena, off, lens)
            st.tx = [bytes(out[int(o) * 64:int(o) * 64 + int(n)]) for o, n in zip(off, lens)]
            st.sent = getattr(st, "sent", []) + st.tx
            st.tx = []
    return st


@pytest.mark.parametrize("one_burst", [False, True])
def test_c1_cpu_reference_path(one_burst):
    st = run_cpu(one_burst)
    assert b"".join(st.ring) == b"".join(MESSAGES)
    assert st.rows[1][4] == c1.FIN_2                # the child reached FIN_2 (tcp_states.c:98)
    assert [e[2] for e in st.log] == [c1.LISTENING, c1.SYN_RECV] + [c1.ESTABLISHED] * (len(MESSAGES) + 1)
    for f in st.sent:                                # every tx segment verifies (ip_out)
        assert pktgen.ip_checksum_of(f) == 0 and pktgen.tcp_checksum_of(f) == 0
    assert st.sent[0][47] == 0x12                    # SYN|ACK first


@pytest.mark.gpu
@pytest.mark.parametrize("one_burst", [False, True])
def test_c1_through_rxg(engine, one_burst):
    import rxg
    st = c1.Stack()
    st.mirror = engine
    tcb, live = pktgen.table_arrays(st.rows)
    engine.tcb_load(tcb, live)
    engine.arp_disable()
    sent = []
    for burst in c1.peer_script(MESSAGES, one_burst):
        frames = [with_checksums(f) for f in burst]
        recs = engine.rx_burst(frames, rxg.REC16)
        bufs = [C.create_string_buffer(f, max(len(f), 64)) for f in frames]
        addr = {C.addressof(b): i for i, b in enumerate(bufs)}

        def tcpswitch(u, idx, state, tcp, ip, m):
            i = addr[m]
            st.tcpswitch(idx, state, frames[i], int(recs[i]["datalen"]))
            return 0

        def rst(u, ip, tcp):
            st.send_reset(frames[addr[ip - 14]])

        ops = rxg.HandoffOps(None, rxg.HANDOFF_FREE(), rxg.HANDOFF_ARP_IN(), rxg.HANDOFF_GET_MAC(),
                             rxg.HANDOFF_ADD_MAC(), rxg.HANDOFF_SEND_RESET(rst), rxg.HANDOFF_ON_SEGMENT(),
                             rxg.HANDOFF_TCPSWITCH(tcpswitch))
        ptrs = (C.c_void_p * len(bufs))(*[C.addressof(b) for b in bufs])
        lib = rxg.load_library()
        assert lib.rxg_rx_replay(engine.ctx, C.byref(ops), ptrs, ptrs, recs.ctypes.data, len(bufs), 16) == 0
        if st.tx:   # ip_out's checksums on the GPU (rxg_tx_cksum_dev)
            arena, off, lens = pktgen.pack_arena(st.tx)
            out = engine.tx_arena(arena, off, lens)
            sent += [bytes(out[int(o) * 64:int(o) * 64 + int(n)]) for o, n in zip(off, lens)]
            st.tx = []
    ref = run_cpu(one_burst)
    assert b"".join(st.ring) == b"".join(MESSAGES)
    assert st.log == ref.log and st.rows == ref.rows
    assert sent == ref.sent                          # byte-identical tx segments
    assert np.all([pktgen.tcp_checksum_of(f) == 0 for f in sent])
