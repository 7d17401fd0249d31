"""TEST INFRASTRUCTURE ONLY — ctypes binding of the CPU oracle (rxg_oracle.c).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this
package, and only as the checker (or the timed CPU baseline), never as a product path.
See rxg_oracle.h for what the oracle restates and how its parity is pinned.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
NCOUNTERS = 16

_REC16 = np.dtype([("tcb_idx", "<i4"), ("ip_cksum", "<u2"), ("tcp_cksum", "<u2"),
                   ("verdict", "u1"), ("state", "u1"), ("tcp_flags", "u1"), ("flags", "u1"),
                   ("datalen", "<i4")])
REC48_DTYPE = np.dtype([("c", _REC16), ("ether_type", "<u2"), ("sport", "<u2"),
                        ("dport", "<u2"), ("l4_proto", "u1"), ("version_ihl", "u1"),
                        ("seq", "<u4"), ("ack", "<u4"), ("src_ip", "<u4"),
                        ("dst_ip_raw", "<u4"), ("data_off", "u1"), ("src_mac", "u1", (6,)),
                        ("reserved", "u1")])
TCB_DTYPE = np.dtype([("dport", "<i4"), ("sport", "<i4"), ("ipv4_dst", "<u4"),
                      ("ipv4_src", "<u4"), ("state", "u1"), ("pad", "u1"),
                      ("identifier", "<u2")])

_libs: dict[str, C.CDLL] = {}


def build():
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def lib(opt: str = "O2") -> C.CDLL:
    name = "liboracle.so" if opt == "O2" else "liboracle_O0.so"
    if name in _libs:
        return _libs[name]
    path = os.path.join(_HERE, name)
    if not os.path.exists(path):
        build()
    L = C.CDLL(path)
    vp, u32, i32 = C.c_void_p, C.c_uint32, C.c_int32
    L.orc_calculate_checksum.restype = C.c_uint16
    L.orc_calculate_checksum.argtypes = [vp, C.c_int]
    for fn in (L.orc_rx_batch, L.orc_rx_batch_faithful, L.orc_rx_batch_shipped):
        fn.restype = C.c_int
        fn.argtypes = [vp, vp, vp, u32, vp, vp, i32, vp, vp]
    L.orc_tx_cksum_batch.restype = C.c_int
    L.orc_tx_cksum_batch.argtypes = [vp, vp, vp, u32]
    L.orc_arp_reset.restype = None
    L.orc_arp_count.restype = C.c_int
    _libs[name] = L
    return L


def _p(a):
    return None if a is None else a.ctypes.data


def calculate_checksum(data: bytes) -> int:
    """ip.c:44-59 (the caller's odd byte past the end is provided as 0)."""
    buf = (C.c_ubyte * (len(data) + 2)).from_buffer_copy(bytes(data) + b"\0\0")
    return lib().orc_calculate_checksum(buf, len(data))


def rx_batch(arena, off64, lens, tcbs, live=None, faithful=False, opt="O2", shipped=False):
    """Records (REC48_DTYPE) and counters (u64[16]) for a packed batch.  shipped (timing only,
    with faithful): the reference as shipped, without the rx checksum verify."""
    n = len(lens)
    arena = np.ascontiguousarray(arena, dtype=np.uint8)
    off64 = np.ascontiguousarray(off64, dtype=np.uint32)
    lens = np.ascontiguousarray(lens, dtype=np.uint16)
    tcbs = np.ascontiguousarray(tcbs, dtype=TCB_DTYPE)
    live = (np.ones(len(tcbs), dtype=np.uint8) if live is None
            else np.ascontiguousarray(live, dtype=np.uint8))
    out = np.zeros(n, dtype=REC48_DTYPE)
    cnt = np.zeros(NCOUNTERS, dtype=np.uint64)
    fn = (lib(opt).orc_rx_batch_shipped if shipped else lib(opt).orc_rx_batch_faithful) if faithful \
        else lib(opt).orc_rx_batch
    fn(_p(arena), _p(off64), _p(lens), n, _p(tcbs) if len(tcbs) else None,
       _p(live) if len(live) else None, len(tcbs), _p(out), _p(cnt))
    return out, cnt


def tx_batch(arena, off64, lens):
    """ip_out's checksums written into a copy of the arena."""
    a = np.array(arena, dtype=np.uint8, copy=True)
    lib().orc_tx_cksum_batch(_p(a), _p(np.ascontiguousarray(off64, dtype=np.uint32)),
                             _p(np.ascontiguousarray(lens, dtype=np.uint16)), len(lens))
    return a


def arp_reset():
    lib().orc_arp_reset()
    lib("O0").orc_arp_reset()


def arp_count(opt: str = "O0") -> int:
    """Entries in the faithful path's ARP list (arp.c:282-317 add_mac) of the given build."""
    return int(lib(opt).orc_arp_count())
