"""CPU: the receive-window restatement (oracle/window.py, tcp_windows.c) branch by branch —
the checker rxg's payload hand-off is compared against."""
import pytest

from oracle import window as W

ACK_PSH, FIN_ACK = 0x18, 0x11


def seg(payload: bytes, doff: int = 5) -> bytes:
    """frame[34:] of a segment: a TCP header of doff words, then the payload."""
    return bytes([0] * 12) + bytes([doff << 4]) + bytes(doff * 4 - 13) + payload


def fresh(cur=1001):
    w = W.ReceiveWindow(4000, 4000)
    w.cur = cur
    return w


def test_in_order_one_message_per_segment():
    w, msgs = fresh(), []
    assert W.push_data(w, 1001, 5, seg(b"hello"), 0x50, ACK_PSH, msgs) == (0, 1006)
    assert W.push_data(w, 1006, 3, seg(b"abc"), 0x50, ACK_PSH, msgs) == (0, 1009)
    assert msgs == [b"hello", b"abc"] and w.cur == 1009 and not w.pairs and w.freed == 2


def test_tcp_options_shift_the_payload():
    w, msgs = fresh(), []
    W.push_data(w, 1001, 4, seg(b"data", doff=8), 0x80, ACK_PSH, msgs)
    assert msgs == [b"data"]


def test_fin_counts_in_ack_not_in_cur():
    w, msgs = fresh(), []
    assert W.push_data(w, 1001, 2, seg(b"ok"), 0x50, FIN_ACK, msgs) == (0, 1004)
    assert msgs == [b"ok"] and w.cur == 1003
    w2, m2 = fresh(), []
    assert W.push_data(w2, 1001, 0, seg(b""), 0x50, FIN_ACK, m2) == (0, 1002)   # bare FIN
    assert m2 == [] and w2.cur == 1001


def test_reordered_segment_is_held_and_the_gap_filler_dropped():
    # the later segment waits as a pair; the in-order one then fails the inverted
    # out-of-window test (seq - first + Length < CurrentSize, tcp_windows.c:345)
    w, msgs = fresh(), []
    assert W.push_data(w, 1011, 5, seg(b"later"), 0x50, ACK_PSH, msgs) == (0, 1016)
    assert msgs == [] and len(w.pairs) == 1 and w.cur == 1001
    assert W.push_data(w, 1001, 10, seg(b"0123456789"), 0x50, ACK_PSH, msgs) == (-1, None)
    assert msgs == [] and len(w.pairs) == 1


def test_duplicates():
    w, msgs = fresh(), []
    W.push_data(w, 1001, 10, seg(b"0123456789"), 0x50, ACK_PSH, msgs)
    assert W.push_data(w, 991, 5, seg(b"old.."), 0x50, ACK_PSH, msgs) == (-1, None)  # cur > seq+len
    # a retransmission ending exactly at cur passes the test, AdjustPair + GetData hand out 0 bytes
    assert W.push_data(w, 1001, 10, seg(b"0123456789"), 0x50, ACK_PSH, msgs) == (0, 1011)
    assert msgs == [b"0123456789"] and w.cur == 1011 and not w.pairs


def test_partial_overlap_delivers_the_new_bytes():
    w, msgs = fresh(), []
    W.push_data(w, 1001, 4, seg(b"abcd"), 0x50, ACK_PSH, msgs)
    W.push_data(w, 1003, 6, seg(b"cdefgh"), 0x50, ACK_PSH, msgs)   # offset 2 into the pair
    assert msgs == [b"abcd", b"efgh"] and w.cur == 1009


def test_sequence_wrap_u32():
    w, msgs = fresh(0xFFFFFFF0), []
    assert W.push_data(w, 0xFFFFFFF0, 32, seg(bytes(range(32))), 0x50, ACK_PSH, msgs) == (-1, None)
    # (seq + Length) wraps to 0x10 < cur: the duplicate test drops it (u32 compare)
    assert msgs == []


def test_reference_asserts():
    with pytest.raises(W.RefAbort, match="< 1000"):
        W.push_data(fresh(), 1001, 1000, seg(bytes(1000)), 0x50, ACK_PSH, [])
    msgs = []
    W.push_data(fresh(), 1001, 1000, seg(bytes(1000)), 0x50, ACK_PSH, msgs, oversize_ok=True)
    assert len(msgs[0]) == 1000
    with pytest.raises(W.RefAbort, match="CurrentSequenceNumber != 0"):
        W.push_data(fresh(0), 0, 4, seg(b"abcd"), 0x50, ACK_PSH, [])
    # a pair covering the last one is deleted and AdjustPair walks off the list's end
    w = fresh()
    W.push_data(w, 5001, 5000, seg(bytes(5000)), 0x50, ACK_PSH, [])
    with pytest.raises(W.RefAbort, match="NULL"):
        W.push_data(w, 6001, 3000, seg(bytes(3000)), 0x50, ACK_PSH, [])
