"""TEST INFRASTRUCTURE ONLY — CPU restatement of the reference's receive window and its
payload hand-off (tcp_ip_stack/tcp_windows.c), the checker for rxg's payload gather
(SURVEY.md §8(f) row 4).  Only tests/ use it: as the checker, and as the "stack's own
PushData" that a test stack runs when rxg_payload_take refuses a segment.

Restated, in the reference's order and arithmetic (u32 sequence numbers, u16 Length):
  PushData          tcp_windows.c:341-358
  AdjustPair        tcp_windows.c:42-110 (pair list kept sorted by insertion rule)
  PushDataInQueue   tcp_windows.c:112-136 (one GetData per PushData)
  GetData           tcp_windows.c:138-186
  DeletePair        tcp_windows.c:32-38  (frees the pair's mbuf)
Window init: AllocReceiveWindow(4000, 4000) for passively opened TCBs (tcp_states.c:155,
tcp_windows.c:371-380); CurrentSequenceNumber = SYN seq + 1 (tcp_states.c:182).

The reference's assert() calls (-O0 build, asserts on) and its NULL dereferences raise
RefAbort here.  The socket ring (rte_ring of 1024, tcp_tcb.c:62) is modelled as unbounded:
the application is assumed to drain it (socket_read, socket_interface.c:277-292).

Parity is pinned by the reference's code only (it has no tests for this path): the
restatement is line-by-line and the tests exercise each branch (in order, reordered,
duplicate, FIN, out-of-window drop, oversize assert).
"""
from __future__ import annotations

from dataclasses import dataclass, field

M32 = 0xFFFFFFFF
FIN = 0x01
GETDATA_BUFFER = 1000  # PushDataInQueue's unsigned char Buffer[1000] (tcp_windows.c:114)


class RefAbort(RuntimeError):
    """The reference would abort (assert) or crash (NULL dereference) here."""


@dataclass
class Pair:  # struct OutOfSeqPair, tcp_windows.h:27-35
    seq: int
    length: int
    payload: bytes  # the mbuf's bytes from frame + 34 + tcp_len (what GetData reads)
    tcp_len: int
    has_fin: int
    flags: int


@dataclass
class ReceiveWindow:  # tcp_windows.h:37-44
    max_size: int = 4000
    current_size: int = 4000
    start_seq: int = 0
    cur: int = 0  # CurrentSequenceNumber
    pairs: list = field(default_factory=list)  # SeqPairs, in list order
    freed: int = 0  # mbufs freed by DeletePair


def adjust_pair(w: ReceiveWindow, seq: int, length: int, payload: bytes, tcp_len: int,
                tcp_flags: int) -> int:
    """tcp_windows.c:42-110.  Returns the 'maximum contiguous data' value (-> ptcb->ack)."""
    # insert after the last pair whose SequenceNumber <= seq (:47-67)
    k = 0
    while k < len(w.pairs) and w.pairs[k].seq <= seq:
        k += 1
    w.pairs.insert(k, Pair(seq, length, payload, tcp_len, tcp_flags & FIN, tcp_flags & FIN))
    # delete extra pairs (:71-103)
    i = 0
    while i < len(w.pairs) and i + 1 < len(w.pairs):
        p, nx = w.pairs[i], w.pairs[i + 1]
        if not p.seq < nx.seq:  # assert(Pair->SequenceNumber < NextPair->SequenceNumber)
            raise RefAbort("AdjustPair: assert(Pair->SequenceNumber < NextPair->SequenceNumber)")
        if ((p.seq + p.length) & M32) >= ((nx.seq + nx.length) & M32):
            del w.pairs[i + 1]  # Pair->Next = NextPair->Next; DeletePair(NextPair)
            w.freed += 1
            # PrePair = Pair; Pair = Pair->Next; NextPair = Pair->Next (:100-102)
            if i + 1 >= len(w.pairs):
                raise RefAbort("AdjustPair: NULL Pair dereferenced after deleting the last pair")
            i += 1
        else:
            i += 1
    head = w.pairs[0]
    return (head.seq + head.length + (1 if head.has_fin else 0)) & M32


def get_data(w: ReceiveWindow, buf_len: int = GETDATA_BUFFER) -> bytes:
    """tcp_windows.c:138-186: at most one pair per call.  Returns the bytes handed out."""
    if w.cur == 0:
        raise RefAbort("GetData: assert(Window->CurrentSequenceNumber != 0)")
    if not w.pairs:
        raise RefAbort("GetData: Pair->mbuf dereferenced with SeqPairs == NULL")
    p = w.pairs[0]
    if p.seq <= w.cur:
        out = b""
        if p.length != 0:
            if not ((p.seq + p.length) & M32) >= w.cur:
                raise RefAbort("GetData: assert(SequenceNumber + Length >= CurrentSequenceNumber)")
            offset = (w.cur - p.seq) & M32
            n = (p.length - offset) & M32
            if not n < buf_len:  # assert((Pair->Length - offset) < len)
                raise RefAbort(f"GetData: assert((Length - offset) < {buf_len}), Length={p.length}")
            out = p.payload[offset:offset + n]
        elif p.flags == 0:
            raise RefAbort("GetData: assert(Pair->Flags != 0) for a zero-length pair")
        w.pairs.pop(0)
        w.cur = (p.seq + p.length) & M32
        w.freed += 1
        return out
    return b""


def push_data(w: ReceiveWindow, seq: int, length: int, seg: bytes, data_off: int,
              tcp_flags: int, messages: list, *, oversize_ok: bool = False):
    """tcp_windows.c:341-358 + PushDataInQueue (:112-136).  length is PushData's uint16_t
    Length; seg = the frame from byte 34 (the TCP header as the reference addresses it,
    whatever the IHL); the payload GetData copies starts tcp_len bytes into it (:164-166).
    Appends the socket-ring message (if any) to `messages`.  Returns (rc, ack): rc -1 =
    dropped (the caller frees the mbuf, tcp_states.c:124-127), ack None then.
    oversize_ok: deliver a message GetData would assert on (rxg's documented behaviour)."""
    length &= 0xFFFF
    if w.pairs and ((seq - w.pairs[0].seq + length) & M32) < w.current_size:
        return -1, None  # "Out of window data, dropping all"
    if w.cur > ((seq + length) & M32):
        return -1, None  # "duplicate packet"
    tcp_len = (data_off >> 4) * 4
    ack = adjust_pair(w, seq, length, bytes(seg[tcp_len:tcp_len + length]), tcp_len, tcp_flags)
    msg = get_data(w, 1 << 32 if oversize_ok else GETDATA_BUFFER)
    if msg:
        messages.append(msg)
    return 0, ack
