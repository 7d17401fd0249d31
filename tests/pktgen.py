"""Frame builders and seeded parity-case generators for the rxg tests.

Frames are built byte by byte from the wire formats (RFC 791/793, the DPDK 2.2 packed
ether_hdr/ipv4_hdr/tcp_hdr the reference reads), with an independent pure-Python RFC 1071
checksum, so the oracle is cross-checked by a second restatement.
"""
from __future__ import annotations

import random
import struct

import numpy as np

LISTENING, ESTABLISHED = 1, 4


def py_checksum(data: bytes) -> int:
    """RFC 1071 one's-complement checksum (= reference calculate_checksum, ip.c:44-59,
    with the odd tail padded by a zero byte)."""
    if len(data) % 2:
        data = data + b"\0"
    s = sum(struct.unpack(f">{len(data) // 2}H", data)) if data else 0
    while s >> 16:
        s = (s & 0xFFFF) + (s >> 16)
    return (~s) & 0xFFFF


def ip4(a, b, c, d) -> int:
    return (a << 24) | (b << 16) | (c << 8) | d


def raw_of_host(ip_host: int) -> int:
    """The reference's u32 view of a network-order address on x86 (ip->dst_addr)."""
    return int.from_bytes(ip_host.to_bytes(4, "big"), "little")


def frame(*, src_ip=ip4(10, 0, 0, 1), dst_ip=ip4(192, 168, 78, 2), sport=1024, dport=80,
          seq=1, ack=1, flags=0x10, payload=b"", ihl=5, doff=5, proto=6, ethertype=0x0800,
          total_length=None, ttl=64, ip_id=0, valid_ip=True, valid_tcp=True,
          src_mac=b"\x02\x00\x0a\x00\x00\x01", dst_mac=b"\x02\x00\xc0\xa8\x4e\x02",
          ip_opts=None, tcp_opts=None) -> bytes:
    """Ethernet II + IPv4 + TCP.  The reference reads TCP at +34 regardless of IHL
    (tcp_in.c:42-45), so IP options shift nothing it reads; they are simply bytes."""
    ip_opts = ip_opts if ip_opts is not None else b"\0" * max(0, (ihl - 5) * 4)
    tcp_opts = tcp_opts if tcp_opts is not None else b"\0" * max(0, (doff - 5) * 4)
    eth = dst_mac + src_mac + struct.pack(">H", ethertype)
    tcp_wo = struct.pack(">HHIIBBHHH", sport, dport, seq & 0xFFFFFFFF, ack & 0xFFFFFFFF,
                         (doff & 0xF) << 4, flags, 0xFFFF, 0, 0) + tcp_opts
    body = tcp_wo + payload
    tl = (20 + len(ip_opts) + len(body)) if total_length is None else total_length
    iph = struct.pack(">BBHHHBBH4s4s", (4 << 4) | (ihl & 0xF), 0, tl & 0xFFFF, ip_id & 0xFFFF,
                      0x4000, ttl, proto, 0, src_ip.to_bytes(4, "big"), dst_ip.to_bytes(4, "big"))
    if valid_ip:
        ck = py_checksum(iph)
        iph = iph[:10] + struct.pack(">H", ck) + iph[12:]
    f = bytearray(eth + iph + ip_opts + body)
    if valid_tcp:
        # the rx verify's definition: pseudo || frame[34 .. 14+total_length) (clamped)
        f[50:52] = b"\0\0"
        ck = tcp_checksum_of(bytes(f))
        f[50:52] = struct.pack(">H", ck)
    return bytes(f)


def tcp_checksum_of(f: bytes) -> int:
    """rx verify definition on a frame, bytes past len read as 0."""
    g = f + b"\0" * max(0, 54 - len(f))
    tl = struct.unpack(">H", g[16:18])[0]
    seglen = max(0, tl - 20)
    seg = (f[34:34 + seglen] if len(f) > 34 else b"")
    seg = seg + b"\0" * (seglen - len(seg))
    pseudo = g[26:34] + b"\x00\x06" + struct.pack(">H", (tl - 20) & 0xFFFF)
    return py_checksum(pseudo + seg)


def ip_checksum_of(f: bytes) -> int:
    g = f + b"\0" * max(0, 54 - len(f))
    return py_checksum(g[14:34])


# ----------------------------------------------------------------------- parity sets ---

def parity_table(rng: random.Random, nflows: int = 200):
    """A TCB table exercising every findtcb quirk (tcp_tcb.c:127-173):
    listeners (incl. one behind a removed slot), duplicate tuples (lowest index wins),
    removed slots, a LISTENING slot with a full tuple, int ports outside 0..65535, an
    active-open TCB holding ipv4_dst in host order (tcp_states.c:27), all states."""
    dst = ip4(192, 168, 78, 2)
    rows, flows = [], []
    rows.append((80, 0, raw_of_host(dst), 0, LISTENING))          # 0: listener :80
    for f in range(nflows):
        src = ip4(10, (f >> 16) & 255, (f >> 8) & 255, f & 255)
        sport = 1024 + f % 64511
        st = ESTABLISHED if f % 7 else rng.randrange(0, 7)
        rows.append((80, sport, raw_of_host(dst), src, st))
        flows.append((src, sport, 80))
    rows.append(None)                                              # removed slot
    rows.append((8080, 0, raw_of_host(dst), 0, LISTENING))         # listener :8080 after NULL
    rows.append(rows[5])                                           # duplicate of slot 5
    rows.append((443, 4242, raw_of_host(dst), ip4(10, 9, 9, 9), LISTENING))  # listening w/ tuple
    rows.append((-1, 5000, raw_of_host(dst), ip4(10, 8, 8, 8), ESTABLISHED))  # bad int port
    rows.append((70000, 5001, raw_of_host(dst), ip4(10, 8, 8, 9), ESTABLISHED))
    rows.append((80, 6000, dst, ip4(10, 7, 7, 7), ESTABLISHED))    # host-order dst (active open)
    rows.append(None)
    rows.append((22, 0, raw_of_host(dst), 0, LISTENING))
    special = {"dup": (rows[5][3], rows[5][1], 80), "listen_tuple": (ip4(10, 9, 9, 9), 4242, 443),
               "badport": (ip4(10, 8, 8, 8), 5000, 65535), "hostdst": (ip4(10, 7, 7, 7), 6000, 80)}
    return rows, flows, special


def random_frame(rng: random.Random, flows, special) -> bytes:
    """One frame from a mixture of valid traffic and every malformed/edge case the path
    meets (short frames, non-IPv4, non-TCP, IHL != 5, odd lengths)."""
    k = rng.random()
    dst = ip4(192, 168, 78, 2)

    def plen():
        r = rng.random()
        if r < 0.3:
            return rng.randrange(0, 12)
        if r < 0.6:
            return rng.randrange(0, 600)
        if r < 0.9:
            return rng.choice([10, 11, 522, 523, 1446, 1445, 1482, 1483, 1994, 1995, 2000])
        return rng.randrange(0, 9000)

    if k < 0.45:  # established flow, maybe bad checksums, random flags
        src, sport, dport = rng.choice(flows)
        return frame(src_ip=src, dst_ip=dst, sport=sport, dport=dport, seq=rng.getrandbits(32),
                     ack=rng.getrandbits(32), flags=rng.getrandbits(8), payload=rng.randbytes(plen()),
                     valid_ip=rng.random() < 0.9, valid_tcp=rng.random() < 0.9)
    if k < 0.55:  # to a listener, SYN or not
        dport = rng.choice([80, 8080, 22, 443, 9999])
        return frame(src_ip=ip4(172, 16, rng.randrange(256), rng.randrange(256)), dst_ip=dst,
                     sport=rng.randrange(65536), dport=dport,
                     flags=rng.choice([0x02, 0x12, 0x10, 0x01, 0x04, 0x00, 0xFF]),
                     payload=rng.randbytes(plen() % 64))
    if k < 0.60:  # special tuples
        src, sport, dport = special[rng.choice(list(special))]
        return frame(src_ip=src, dst_ip=dst, sport=sport, dport=dport, flags=rng.choice([2, 16]),
                     payload=rng.randbytes(rng.randrange(40)))
    if k < 0.65:  # IHL != 5 / doff != 5 / options
        src, sport, dport = rng.choice(flows)
        ihl, doff = rng.randrange(0, 16), rng.randrange(0, 16)
        return frame(src_ip=src, sport=sport, dport=dport, ihl=ihl, doff=doff,
                     ip_opts=rng.randbytes(max(0, ihl - 5) * 4), tcp_opts=rng.randbytes(max(0, doff - 5) * 4),
                     payload=rng.randbytes(plen() % 200))
    if k < 0.72:  # total_length disagrees with data_len
        src, sport, dport = rng.choice(flows)
        f = frame(src_ip=src, sport=sport, dport=dport, payload=rng.randbytes(plen() % 1500))
        tl = rng.choice([0, 1, 19, 20, 21, 39, 40, 41, rng.randrange(65536), len(f) - 14 + rng.randrange(-30, 30)])
        return f[:16] + struct.pack(">H", tl & 0xFFFF) + f[18:]
    if k < 0.77:  # IPv4, not TCP
        return frame(proto=rng.choice([1, 17, 47, 0, 255]), payload=rng.randbytes(plen() % 300))
    if k < 0.82:  # ARP
        arp = struct.pack(">HHBBH", 1, 0x0800, 6, 4, rng.choice([1, 2])) + rng.randbytes(20)
        return b"\xff" * 6 + rng.randbytes(6) + b"\x08\x06" + arp + b"\0" * rng.randrange(0, 20)
    if k < 0.86:  # other ethertypes
        et = rng.choice([0x86DD, 0x8100, 0x88CC, 0x0000, 0xFFFF, 0x0008])
        return rng.randbytes(12) + struct.pack(">H", et) + rng.randbytes(rng.randrange(0, 200))
    if k < 0.93:  # short / truncated frames (reference reads stale bytes; rxg reads zeros)
        src, sport, dport = rng.choice(flows)
        f = frame(src_ip=src, sport=sport, dport=dport)
        return f[:rng.randrange(0, 54)]
    # pure noise with an IPv4 ethertype
    return rng.randbytes(12) + b"\x08\x00" + rng.randbytes(rng.randrange(0, 2100))


def parity_set(seed: int, n: int, nflows: int = 200):
    rng = random.Random(seed)
    rows, flows, special = parity_table(rng, nflows)
    frames = [random_frame(rng, flows, special) for _ in range(n)]
    return rows, frames


def pack_arena(frames):
    """rxg batch layout: frames at 64-byte aligned starts (see rxg.pack_arena)."""
    n = len(frames)
    lens = np.array([len(f) for f in frames], dtype=np.uint32)
    slots = (lens + 63) // 64
    off = np.zeros(n, dtype=np.uint64)
    if n > 1:
        off[1:] = np.cumsum(slots[:-1])
    arena = np.zeros(max(int(slots.sum()) * 64, 64), dtype=np.uint8)
    for i, f in enumerate(frames):
        o = int(off[i]) * 64
        arena[o:o + len(f)] = np.frombuffer(f, dtype=np.uint8)
        # padding up to the slot end holds garbage: the kernel must ignore it
        pad = int(slots[i]) * 64 - len(f)
        if pad:
            arena[o + len(f):o + len(f) + pad] = 0xA5
    return arena, off.astype(np.uint32), lens.astype(np.uint16)


def table_arrays(rows):
    tcb = np.zeros(len(rows), dtype=[("dport", "<i4"), ("sport", "<i4"), ("ipv4_dst", "<u4"),
                                     ("ipv4_src", "<u4"), ("state", "u1"), ("pad", "u1"),
                                     ("identifier", "<u2")])
    live = np.zeros(len(rows), dtype=np.uint8)
    for i, r in enumerate(rows):
        if r is None:
            continue
        live[i] = 1
        tcb[i] = (r[0], r[1], r[2] & 0xFFFFFFFF, r[3] & 0xFFFFFFFF, r[4], 0, (i % 65535) + 1)
    return tcb, live
