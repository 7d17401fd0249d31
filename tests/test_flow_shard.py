"""Flow-affinity sharding, host side (no GPU): the RSS steering function
(rxg_flow_part_of / rxg_rss_hash).

The Toeplitz hash is pinned by the five IPv4/TCP verification vectors of Microsoft's RSS
specification ("Verifying the RSS Hash Calculation", default 40-byte key), the hash NIC rx
queues are steered by.  The reference (one rx lcore, main.c:366-369) has no RSS of its own.
"""
import ipaddress
import random
import struct

import pytest

import pktgen
import rxg

# (src ip, src port, dst ip, dst port) -> hash over src ip | dst ip | src port | dst port
MS_RSS_TCP_VECTORS = [
    ("66.9.149.187", 2794, "161.142.100.80", 1766, 0x51CCC178),
    ("199.92.111.2", 14230, "65.69.140.83", 4739, 0xC626B0EA),
    ("24.19.198.95", 12898, "12.22.207.184", 38024, 0x5C2B394A),
    ("38.27.205.30", 48228, "209.142.163.6", 2217, 0xAFC7327F),
    ("153.39.163.191", 44251, "202.188.127.2", 1303, 0x10E828A2),
]


def _wire(src, sport, dst, dport):
    return ipaddress.IPv4Address(src).packed + ipaddress.IPv4Address(dst).packed + struct.pack(">HH", sport, dport)


@pytest.mark.parametrize("src,sport,dst,dport,h", MS_RSS_TCP_VECTORS)
def test_rss_hash_known_answers(src, sport, dst, dport, h):
    assert rxg.rss_hash(_wire(src, sport, dst, dport)) == h


def test_flow_part_of_frames():
    """A TCP frame's queue is the RSS hash of its bytes 26..37 through the default
    redirection table (128 entries, entry i -> queue i % n)."""
    for src, sport, dst, dport, h in MS_RSS_TCP_VECTORS:
        f = pktgen.frame(src_ip=int(ipaddress.IPv4Address(src)), dst_ip=int(ipaddress.IPv4Address(dst)),
                         sport=sport, dport=dport, payload=b"x" * 10)
        for n in (1, 2, 3, 4, 8):
            assert rxg.flow_part_of(f, n) == (h % rxg.RSS_RETA_SIZE) % n


def test_flow_part_of_non_tcp_and_truncated():
    f = pktgen.frame(sport=5555, dport=80)
    arp = f[:12] + b"\x08\x06" + f[14:]
    udp = f[:23] + b"\x11" + f[24:]
    for g in (arp, udp, b"", f[:13]):
        assert rxg.flow_part_of(g, 4) == 0
    # truncated TCP frames: the missing bytes read as zero, as the kernel reads them
    for cut in (24, 30, 36, 37):
        g = f[:cut]
        w = (g + bytes(38 - cut))[26:38]
        assert rxg.flow_part_of(g, 8) == (rxg.rss_hash(w) % rxg.RSS_RETA_SIZE) % 8


def test_flow_part_of_rejects_bad_arguments():
    for n in (0, rxg.RSS_RETA_SIZE + 1):
        with pytest.raises(rxg.RxgError):
            rxg.flow_part_of(pktgen.frame(), n)


def test_flow_parts_balance():
    """The parity table's flows spread over the queues (each within 25 % of 1/n)."""
    rng = random.Random(5)
    rows, flows, _ = pktgen.parity_table(rng, 3000)
    for n in (2, 3, 4):
        cnt = [0] * n
        for src, sport, dport in flows:
            cnt[rxg.flow_part_of(pktgen.frame(src_ip=src, sport=sport, dport=dport), n)] += 1
        assert min(cnt) > 0.75 * len(flows) / n, cnt


def test_flow_part_of_table_equals_bitwise_hash():
    """rxg_flow_part_of (byte tables) against rxg_rss_hash (the bit-serial definition) on
    random tuples, through the whole 128-entry redirection table."""
    rng = random.Random(11)
    base = bytearray(pktgen.frame(sport=1, dport=2))
    for _ in range(2000):
        w = rng.randbytes(12)
        base[26:38] = w
        assert rxg.flow_part_of(bytes(base), rxg.RSS_RETA_SIZE) == rxg.rss_hash(w) % rxg.RSS_RETA_SIZE
