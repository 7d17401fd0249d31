"""TEST INFRASTRUCTURE ONLY — CPU restatement of rxg_payload_gather_dev's output, the
checker of the device payload gather.

Which frames carry a payload for the socket ring, and which bytes, follows the reference:
  datalen = ntohs(total_length) - (version_ihl & 0xf)*4 - (data_off >> 4)*4
            (tcp_established, tcp_states.c:103-111; the record's datalen)
  bytes   = frame[34 + (data_off >> 4)*4 : ... + datalen]   (GetData, tcp_windows.c:164-166:
            the IP header is taken as 20 bytes whatever the IHL)
for every TCP segment of the burst (verdicts DISPATCH, RST_NOPCB, RST_LISTEN_NONSYN: the
replay can turn the latter into a DISPATCH when a handler creates the TCB in the burst;
whether PushData is reached and takes the segment is decided at replay time).  Frames
whose payload would run past the frame (the reference copies stale mbuf bytes there),
records marked RXG_F_TRUNC and datalen <= 0 are left to the stack.  Layout (rxg's):
packet order, each message 16-byte aligned and zero padded; frames past the arena
capacity are not gathered.  slots(): the same messages as rxg_rx_burst_payload_dev lays them
out (the fused burst + hand-off: each payload stays at its frame's offset in the pool).
"""
from __future__ import annotations

import numpy as np

V_RST_LISTEN_NONSYN = 2
F_TRUNC = 0x10
PM_GATHERED, PM_REF_OVERSIZE = 0x01, 0x02
MSG_DTYPE = np.dtype([("arena_off", "<u8"), ("len", "<u4"), ("flags", "<u4")])


def candidate(frame: bytes, rec) -> bytes | None:
    """rec: an rxg_rec16-shaped record (fields verdict, flags, datalen)."""
    datalen = int(rec["datalen"])
    if int(rec["verdict"]) > V_RST_LISTEN_NONSYN or datalen <= 0 or int(rec["flags"]) & F_TRUNC:
        return None
    start = 34 + (frame[46] >> 4) * 4
    if start + datalen > len(frame):
        return None
    return bytes(frame[start:start + datalen])


def gather(frames, recs, arena_cap: int):
    """Expected (msgs, the gathered messages' arena bytes, bytes needed)."""
    n = len(frames)
    msgs = np.zeros(n, dtype=MSG_DTYPE)
    parts, off = [], 0
    for i, f in enumerate(frames):
        p = candidate(f, recs[i])
        if p is None:
            continue
        r16 = (len(p) + 15) & ~15
        if off + r16 <= arena_cap:
            msgs[i] = (off, len(p), PM_GATHERED | (PM_REF_OVERSIZE if len(p) >= 1000 else 0))
            parts.append(p + b"\0" * (r16 - len(p)))
        off += r16
    return msgs, np.frombuffer(b"".join(parts), dtype=np.uint8), off


def slots(frames, recs, off64):
    """Expected messages of rxg_rx_burst_payload_dev: the candidates of gather(), each at its
    offset in the frame pool (arena_off = 64 * off64[i] + 34 + data_off * 4), same len and
    flags; returns (msgs, [payload bytes or None per frame])."""
    n = len(frames)
    msgs = np.zeros(n, dtype=MSG_DTYPE)
    pays = []
    for i, f in enumerate(frames):
        p = candidate(f, recs[i])
        pays.append(p)
        if p is None:
            continue
        start = 34 + (f[46] >> 4) * 4
        msgs[i] = (int(off64[i]) * 64 + start, len(p), PM_GATHERED | (PM_REF_OVERSIZE if len(p) >= 1000 else 0))
    return msgs, pays
