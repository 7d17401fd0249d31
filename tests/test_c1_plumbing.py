"""Config 1 (plumbing): socket_tester-style listener <-> scripted samplesocketclient peer,
one TCP flow, handshake -> data -> FIN.  The CPU test runs the reference rx path (the
oracle, one packet at a time) and the reference receive window (oracle/window.py) — no
GPU; the GPU test runs the same exchange through rxg (burst + device payload gather +
in-order replay + tx checksum generate) and must produce the same bytes."""
import pytest

import c1_stack as c1
import pktgen

# (payloads < 1000 bytes: GetData asserts on larger ones, tcp_windows.c:170)
MESSAGES = [b"Hello World %d" % i for i in range(5)] + [bytes(range(256)) * 3 + bytes(range(200))]


@pytest.mark.parametrize("one_burst", [False, True])
def test_c1_cpu_reference_path(one_burst):
    st = c1.drive_cpu(c1.peer_script(MESSAGES, one_burst))
    assert st.ring == MESSAGES                       # one socket-ring message per segment
    assert st.rows[1][4] == c1.FIN_2                 # the child reached FIN_2 (tcp_states.c:98)
    assert [e[2] for e in st.log] == [c1.LISTENING, c1.SYN_RECV] + [c1.ESTABLISHED] * (len(MESSAGES) + 1)
    for f in st.sent:                                # every tx segment verifies (ip_out)
        assert pktgen.ip_checksum_of(f) == 0 and pktgen.tcp_checksum_of(f) == 0
    assert st.sent[0][47] == 0x12                    # SYN|ACK first
    assert st.tcb[1]["ack"] == 1001 + sum(map(len, MESSAGES)) + 1   # AdjustPair + FIN


@pytest.mark.gpu
@pytest.mark.parametrize("one_burst", [False, True])
def test_c1_through_rxg(engine, one_burst):
    st = c1.drive_rxg(engine, c1.peer_script(MESSAGES, one_burst))
    ref = c1.drive_cpu(c1.peer_script(MESSAGES, one_burst))
    assert st.ring == MESSAGES
    assert st.log == ref.log and st.rows == ref.rows
    assert st.sent == ref.sent                       # byte-identical tx segments
    assert {i: t["ack"] for i, t in st.tcb.items()} == {i: t["ack"] for i, t in ref.tcb.items()}
    # every data segment's payload comes from the device gather (in one burst the segments
    # classify to the listener before the replay creates the child, and are gathered anyway)
    assert st.taken == len(MESSAGES)


@pytest.mark.gpu
def test_c1_per_packet_ether_in(engine):
    """ether_in(m) per mbuf, unchanged call site, each call a GPU burst of one."""
    st = c1.drive_rxg_per_packet(engine, c1.peer_script(MESSAGES, True))
    ref = c1.drive_cpu(c1.peer_script(MESSAGES, True))
    assert st.ring == MESSAGES
    assert st.log == ref.log and st.rows == ref.rows and st.sent == ref.sent
