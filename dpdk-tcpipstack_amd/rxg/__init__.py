"""rxg — Python binding of the MI355X receive-path engine's C ABI (include/rxg.h).

This is a thin ctypes layer used by tests/, bench.py and __graft_entry__.py; the engine
itself is librxg.so (HIP kernels for gfx950 + C++ host code).  There is no Python or CPU
compute path: if librxg.so is missing, or no GPU is present, calls raise RxgError.

The reference surface this mirrors (rajneshrat/dpdk-tcpipstack, tcp_ip_stack/):
  ether_in/ip_in/tcp_in/findtcb per packet    -> Engine.rx_burst_dev / Engine.rx_burst
  tcbs[] writes (alloc_tcb, remove_tcb, state) -> Engine.tcb_upsert / tcb_remove / tcb_set_state
  ip_out's two checksums (ip.c:97-118)        -> Engine.tx_cksum_dev
"""
from __future__ import annotations

import ctypes as C
import os
import sys

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_PRODUCT_LIB = os.path.join(_HERE, "librxg.so")
# RXG_LIB swaps in another build (an experiment or an older library for an A/B) only with
# the explicit opt-in RXG_LIB_OVERRIDE=1: a stray RXG_LIB must not put another library under
# the tests, smoke() or bench.py.  load_library() refuses it otherwise.
LIB_PATH = os.environ.get("RXG_LIB") or _PRODUCT_LIB


def source_hash(root: str = os.path.dirname(_HERE)) -> str:
    """The product sources' hash exactly as the Makefile compiles it into rxg_build_info
    (src=...): sha256 over csrc/*.h, *.hip, *.cpp in sorted order, then include/rxg.h."""
    import glob
    import hashlib
    csrc = os.path.join(root, "csrc")
    files = sorted(os.path.relpath(p, root) for ext in ("h", "hip", "cpp")
                   for p in glob.glob(os.path.join(csrc, "*." + ext)))
    h = hashlib.sha256()
    for rel in files + [os.path.join("..", "include", "rxg.h")]:
        with open(os.path.join(root, rel), "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


def build_provenance(lib=None) -> dict:
    """What the loaded library says it was built from, and whether that is this tree."""
    lib = lib or load_library()
    info = lib.rxg_build_info().decode()
    src = next((w[4:] for w in info.split() if w.startswith("src=")), None)
    tree = source_hash()
    return {"build": info, "lib": os.path.abspath(_loaded_path or LIB_PATH), "source_hash": tree,
            "build_matches_tree": src == tree}

# ---------------------------------------------------------------- constants (rxg.h) ---
ETHER_TYPE_IPV4 = 0x0800
ETHER_TYPE_ARP = 0x0806
IPPROTO_TCP = 6
TCP_FLAG_FIN, TCP_FLAG_SYN, TCP_FLAG_RST, TCP_FLAG_PSH, TCP_FLAG_ACK = 1, 2, 4, 8, 16
(TCP_STATE_CLOSED, LISTENING, SYN_SENT, SYN_RECV, TCP_ESTABLISHED, TCP_STATE_FIN_1,
 TCP_FIN_2) = range(7)
STATE_NONE = 0xFF

V_DISPATCH, V_RST_NOPCB, V_RST_LISTEN_NONSYN, V_DROP_NONTCP, V_ARP, V_DROP_L2 = range(6)
F_IP_OK, F_TCP_OK, F_LISTEN, F_REF_NULLSLOT, F_TRUNC, F_ARP_LEARN = 1, 2, 4, 8, 16, 32
REC8, REC16, REC48 = 8, 16, 48
# rxg_server_config.flags and rxg_server_placement (include/rxg.h)
SRV_HOST_STAGING = 1
SRV_HOST_MAILBOX = 2
SRV_NONE, SRV_HOST, SRV_DEVICE = 0, 1, 2

COUNTERS = ["rx", "bytes", "ipv4", "arp", "other_l2", "tcp", "non_tcp", "ip_cksum_bad",
            "tcp_cksum_bad", "tcb_hit_exact", "tcb_hit_listen", "nopcb", "listen_nonsyn",
            "dispatch", "ref_nullslot", "trunc"]
NCOUNTERS = len(COUNTERS)

# numpy views of the C records
REC16_DTYPE = np.dtype([("tcb_idx", "<i4"), ("ip_cksum", "<u2"), ("tcp_cksum", "<u2"),
                        ("verdict", "u1"), ("state", "u1"), ("tcp_flags", "u1"),
                        ("flags", "u1"), ("datalen", "<i4")])
REC48_DTYPE = np.dtype([("c", REC16_DTYPE), ("ether_type", "<u2"), ("sport", "<u2"),
                        ("dport", "<u2"), ("l4_proto", "u1"), ("version_ihl", "u1"),
                        ("seq", "<u4"), ("ack", "<u4"), ("src_ip", "<u4"),
                        ("dst_ip_raw", "<u4"), ("data_off", "u1"), ("src_mac", "u1", (6,)),
                        ("reserved", "u1")])
PM_GATHERED, PM_REF_OVERSIZE = 0x01, 0x02
PAYLOAD_MSG_DTYPE = np.dtype([("arena_off", "<u8"), ("len", "<u4"), ("flags", "<u4")])
TCB_DTYPE = np.dtype([("dport", "<i4"), ("sport", "<i4"), ("ipv4_dst", "<u4"),
                      ("ipv4_src", "<u4"), ("state", "u1"), ("pad", "u1"),
                      ("identifier", "<u2")])
assert REC16_DTYPE.itemsize == 16 and REC48_DTYPE.itemsize == 48 and TCB_DTYPE.itemsize == 20
REC8_DTYPE = np.dtype([("w0", "<u4"), ("w1", "<u4")])


def rec8_pack(r16: np.ndarray) -> np.ndarray:
    """rxg_rec16 -> rxg_rec8 (rxg.h): the record the kernel writes for RXG_REC8."""
    out = np.zeros(len(r16), dtype=REC8_DTYPE)
    st = r16["state"].astype(np.uint32)
    st[st == STATE_NONE] = 7
    out["w0"] = (((r16["tcb_idx"].astype(np.int64) + 1) & 0xFFFFFF).astype(np.uint32)
                 | (r16["verdict"].astype(np.uint32) << 24) | (st << 27))
    out["w1"] = (r16["tcp_flags"].astype(np.uint32) | (r16["flags"].astype(np.uint32) << 8)
                 | (((r16["datalen"].astype(np.int64) + 128) & 0x1FFFF).astype(np.uint32) << 14))
    return out


def rec8_expand(r8: np.ndarray) -> np.ndarray:
    """rxg_rec8 -> rxg_rec16 as rxg_rec8_expand (rxg.h) does it: a checksum the record
    knows only as 'not zero' reads 0xFFFF."""
    w0, w1 = r8["w0"].astype(np.uint32), r8["w1"].astype(np.uint32)
    out = np.zeros(len(r8), dtype=REC16_DTYPE)
    v = (w0 >> 24) & 7
    st = (w0 >> 27) & 7
    fl = (w1 >> 8) & 0x3F
    out["tcb_idx"] = (w0 & 0xFFFFFF).astype(np.int32) - 1
    out["ip_cksum"] = np.where((v <= V_DROP_NONTCP) & ((fl & F_IP_OK) == 0), 0xFFFF, 0)
    out["tcp_cksum"] = np.where((v <= V_RST_LISTEN_NONSYN) & ((fl & F_TCP_OK) == 0), 0xFFFF, 0)
    out["verdict"] = v
    out["state"] = np.where(st == 7, STATE_NONE, st)
    out["tcp_flags"] = w1 & 0xFF
    out["flags"] = fl
    out["datalen"] = ((w1 >> 14) & 0x1FFFF).astype(np.int32) - 128
    return out


def rec_dtype(rec_kind: int) -> np.dtype:
    return {REC8: REC8_DTYPE, REC16: REC16_DTYPE, REC48: REC48_DTYPE}[rec_kind]


class RxgError(RuntimeError):
    pass


# ------------------------------------------------------------------- ctypes structs ---
ABI_VERSION = 2
RSS_RETA_SIZE = 128  # rxg.h RXG_RSS_RETA_SIZE: the default redirection table


class Config(C.Structure):
    _fields_ = [("device", C.c_int32), ("max_batch", C.c_uint32), ("max_bytes", C.c_uint32),
                ("flags", C.c_uint32), ("max_blocks", C.c_uint32), ("zc_bytes", C.c_uint32)]


class TcbTuple(C.Structure):
    _fields_ = [("dport", C.c_int32), ("sport", C.c_int32), ("ipv4_dst", C.c_uint32),
                ("ipv4_src", C.c_uint32), ("state", C.c_uint8), ("pad", C.c_uint8),
                ("identifier", C.c_uint16)]


TCB_OP_UPSERT, TCB_OP_REMOVE, TCB_OP_SET_STATE = 1, 2, 3
TCB_QUEUE_CAP = 65536


class TcbOp(C.Structure):
    """rxg_tcb_op (include/rxg.h): a tcbs[] write posted from another thread."""
    _fields_ = [("kind", C.c_uint32), ("idx", C.c_int32), ("tuple", TcbTuple), ("state", C.c_uint8),
                ("pad", C.c_uint8 * 3)]


class DevBatch(C.Structure):
    _fields_ = [("frames", C.c_void_p), ("off64", C.c_void_p), ("len", C.c_void_p),
                ("n", C.c_uint32), ("rec_kind", C.c_uint32), ("out", C.c_void_p)]


class ServerConfig(C.Structure):
    """rxg_server_config: latency mode (rxg_server_start)."""
    _fields_ = [("rec_kind", C.c_uint32), ("blocks", C.c_uint32), ("max_frames", C.c_uint32),
                ("max_bytes", C.c_uint32), ("idle_ms", C.c_uint32), ("flags", C.c_uint32)]


class DevBurst(C.Structure):
    """rxg_dev_burst: one burst of a multi-burst launch (rxg_rx_bursts_dev)."""
    _fields_ = [("off64", C.c_void_p), ("len", C.c_void_p), ("n", C.c_uint32), ("pad", C.c_uint32),
                ("out", C.c_void_p)]


class DevStridedBurst(C.Structure):
    """rxg_dev_strided_burst: one burst of a fixed-stride launch (rxg_rx_bursts_strided_dev)."""
    _fields_ = [("len", C.c_void_p), ("n", C.c_uint32), ("slot0", C.c_uint32), ("out", C.c_void_p)]


class DevTxBatch(C.Structure):
    _fields_ = [("frames", C.c_void_p), ("off64", C.c_void_p), ("len", C.c_void_p),
                ("n", C.c_uint32), ("pad", C.c_uint32)]


class PktView(C.Structure):
    _fields_ = [("buf_addr", C.c_void_p), ("data_off", C.c_uint16), ("data_len", C.c_uint16),
                ("pad", C.c_uint32)]


class PayloadMsg(C.Structure):
    _fields_ = [("arena_off", C.c_uint64), ("len", C.c_uint32), ("flags", C.c_uint32)]


class PayloadOut(C.Structure):
    _fields_ = [("arena", C.c_void_p), ("arena_cap", C.c_uint64), ("msgs", C.c_void_p),
                ("arena_used", C.c_void_p)]


class PayloadSlots(C.Structure):
    """rxg_payload_slots: the fused burst's payload arena (the pool's geometry) and messages."""
    _fields_ = [("arena", C.c_void_p), ("msgs", C.c_void_p)]


class SynthParams(C.Structure):
    _fields_ = [("seed", C.c_uint64), ("n", C.c_uint32), ("nflows", C.c_uint32),
                ("dst_ip_host", C.c_uint32), ("dport", C.c_uint16), ("mix", C.c_uint16),
                ("len_a", C.c_uint16), ("pad", C.c_uint16)]


HANDOFF_FREE = C.CFUNCTYPE(None, C.c_void_p, C.c_void_p)
HANDOFF_ARP_IN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p)
HANDOFF_GET_MAC = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_uint32, C.c_void_p)
HANDOFF_ADD_MAC = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_uint32, C.c_void_p)
HANDOFF_SEND_RESET = C.CFUNCTYPE(None, C.c_void_p, C.c_void_p, C.c_void_p)
HANDOFF_ON_SEGMENT = C.CFUNCTYPE(None, C.c_void_p, C.c_int32, C.c_uint32, C.c_uint32)
HANDOFF_TCPSWITCH = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_int32, C.c_uint8, C.c_void_p,
                                C.c_void_p, C.c_void_p)


class HandoffOps(C.Structure):
    _fields_ = [("user", C.c_void_p), ("free_mbuf", HANDOFF_FREE), ("arp_in", HANDOFF_ARP_IN),
                ("get_mac", HANDOFF_GET_MAC), ("add_mac", HANDOFF_ADD_MAC),
                ("send_reset", HANDOFF_SEND_RESET), ("on_segment", HANDOFF_ON_SEGMENT),
                ("tcpswitch", HANDOFF_TCPSWITCH),
                # tcp_in.c:18-19 globals (int*), bumped by the replay; NULL = not kept
                ("tcpnopcb", C.POINTER(C.c_int)), ("tcpchecksumerror", C.POINTER(C.c_int)),
                ("flags", C.c_uint32)]


OPS_VERIFY_TCP_CKSUM = 0x1  # rxg_handoff_ops.flags: tcp_in.c:37-41 compiled in
CFG_REPLAY_ON_DEVICE = 0x1  # rxg_config.flags: every replay fix-up is a GPU re-classify
CFG_STREAMS_OUTLIVE_WRITES = 0x2  # caller streams stay valid until the next table write


# ------------------------------------------------------------------------- loading ---
_lib = None
_loaded_path = None


def load_library(path: str = LIB_PATH):
    """Load librxg.so.  torch (if installed) is imported first so that librxg binds to the
    same HIP runtime copy torch loaded (one HIP runtime per process)."""
    global _lib, _loaded_path
    if _lib is not None:
        return _lib
    if os.path.abspath(path) != _PRODUCT_LIB and os.environ.get("RXG_LIB_OVERRIDE") != "1":
        raise RxgError(f"refusing to load {path} in place of the product library {_PRODUCT_LIB}: "
                       "set RXG_LIB_OVERRIDE=1 as well to load another build")
    if not os.path.exists(path):
        raise RxgError(f"librxg.so not built: {path} (run __graft_entry__.build())")
    if "torch" not in sys.modules:
        try:
            import torch  # noqa: F401
        except Exception:  # pragma: no cover - torch is optional for the binding
            pass
    lib = C.CDLL(path)
    vp, u32, i32, u64 = C.c_void_p, C.c_uint32, C.c_int32, C.c_uint64
    sig = {
        "rxg_abi_version": (C.c_int, []),
        "rxg_build_info": (C.c_char_p, []),
        "rxg_last_error": (C.c_char_p, []),
        "rxg_init": (C.c_int, [C.POINTER(Config), C.POINTER(vp)]),
        "rxg_fini": (C.c_int, [vp]),
        "rxg_sync": (C.c_int, [vp]),
        "rxg_stream": (vp, [vp]),
        "rxg_stream_register": (C.c_int, [vp, vp]),
        "rxg_stream_retire": (C.c_int, [vp, vp]),
        "rxg_tcb_upsert": (C.c_int, [vp, i32, C.POINTER(TcbTuple)]),
        "rxg_tcb_remove": (C.c_int, [vp, i32]),
        "rxg_tcb_set_state": (C.c_int, [vp, i32, C.c_uint8]),
        "rxg_tcb_load": (C.c_int, [vp, vp, vp, i32]),
        "rxg_tcb_sync": (C.c_int, [vp]),
        "rxg_tcb_count": (i32, [vp]),
        "rxg_flow_partition": (C.c_int, [vp, u32, u32]),
        "rxg_flow_partition_get": (C.c_int, [vp, C.POINTER(u32), C.POINTER(u32)]),
        "rxg_flow_part_of": (C.c_int, [C.c_char_p, u32, u32]),
        "rxg_rss_hash": (u32, [C.c_char_p]),
        "rxg_tcb_keys": (C.c_int64, [vp]),
        "rxg_tcb_post": (C.c_int, [vp, C.POINTER(TcbOp)]),
        "rxg_tcb_drain": (C.c_int, [vp]),
        "rxg_arp_load": (C.c_int, [vp, vp, u32]),
        "rxg_arp_learned": (C.c_int, [vp, u32]),
        "rxg_arp_count": (i32, [vp]),
        "rxg_arp_disable": (C.c_int, [vp]),
        "rxg_rx_burst_dev": (C.c_int, [vp, C.POINTER(DevBatch), vp]),
        "rxg_rx_bursts_dev": (C.c_int, [vp, vp, vp, u32, u32, vp]),
        "rxg_rx_bursts_strided_dev": (C.c_int, [vp, vp, u32, vp, u32, u32, vp]),
        "rxg_rx_burst": (C.c_int, [vp, C.POINTER(PktView), u32, u32, vp]),
        "rxg_tx_cksum_dev": (C.c_int, [vp, C.POINTER(DevTxBatch), vp]),
        "rxg_server_start": (C.c_int, [vp, C.POINTER(ServerConfig)]),
        "rxg_server_placement": (C.c_int, [vp]),
        "rxg_server_stop": (C.c_int, [vp]),
        "rxg_server_active": (C.c_int, [vp]),
        "rxg_server_burst_dev": (C.c_int, [vp, C.POINTER(DevBatch)]),
        "rxg_counters_reset": (C.c_int, [vp, vp]),
        "rxg_counters_read": (C.c_int, [vp, vp]),
        "rxg_counters_dev": (vp, [vp]),
        "rxg_rx_replay": (C.c_int, [vp, C.POINTER(HandoffOps), vp, vp, vp, u32, u32]),
        "rxg_ether_in": (C.c_int, [vp, C.POINTER(HandoffOps), vp, vp, C.c_uint16]),
        "rxg_replay_stats": (C.c_int, [vp, vp]),
        "rxg_payload_gather_dev": (C.c_int, [vp, C.POINTER(PayloadOut), vp]),
        "rxg_rx_burst_payload_dev": (C.c_int, [vp, C.POINTER(DevBatch), C.POINTER(PayloadSlots), vp]),
        "rxg_rx_burst_strided_payload_dev": (C.c_int, [vp, vp, u32, C.POINTER(DevStridedBurst), u32,
                                                       C.POINTER(PayloadSlots), vp]),
        "rxg_rcv_set": (C.c_int, [vp, i32, u32, u32]),
        "rxg_payload_take": (C.c_int, [vp, i32, u32, u32, C.POINTER(PayloadMsg)]),
        "rxg_synth_dev": (C.c_int, [vp, C.POINTER(SynthParams), vp, u64, vp, vp, vp,
                                    C.POINTER(u64), vp]),
        "rxg_synth_arena_bytes": (u64, [C.POINTER(SynthParams)]),
        "rxg_dev_alloc": (C.c_int, [vp, u64, C.POINTER(vp)]),
        "rxg_dev_free": (C.c_int, [vp, vp]),
        "rxg_host_alloc_pinned": (C.c_int, [vp, u64, C.POINTER(vp)]),
        "rxg_host_free_pinned": (C.c_int, [vp, vp]),
        "rxg_host_register": (C.c_int, [vp, vp, u64, C.POINTER(vp)]),
        "rxg_host_unregister": (C.c_int, [vp, vp]),
        "rxg_memcpy_h2d": (C.c_int, [vp, vp, vp, u64, vp]),
        "rxg_memcpy_d2h": (C.c_int, [vp, vp, vp, u64, vp]),
        "rxg_memset_dev": (C.c_int, [vp, vp, C.c_int, u64, vp]),
        "rxg_stream_sync": (C.c_int, [vp, vp]),
        "rxg_event_create": (C.c_int, [vp, C.POINTER(vp)]),
        "rxg_event_record": (C.c_int, [vp, vp, vp]),
        "rxg_event_elapsed_ms": (C.c_int, [vp, vp, vp, C.POINTER(C.c_float)]),
        "rxg_event_destroy": (C.c_int, [vp, vp]),
        "rxg_group_init": (C.c_int, [vp, u32, C.POINTER(Config), C.POINTER(vp)]),
        "rxg_group_fini": (C.c_int, [vp]),
        "rxg_group_size": (u32, [vp]),
        "rxg_group_member": (vp, [vp, u32]),
        "rxg_group_tcb_upsert": (C.c_int, [vp, i32, C.POINTER(TcbTuple)]),
        "rxg_group_tcb_remove": (C.c_int, [vp, i32]),
        "rxg_group_tcb_set_state": (C.c_int, [vp, i32, C.c_uint8]),
        "rxg_group_tcb_load": (C.c_int, [vp, vp, vp, i32]),
        "rxg_group_tcb_post": (C.c_int, [vp, C.POINTER(TcbOp)]),
        "rxg_group_tcb_drain": (C.c_int, [vp]),
        "rxg_group_arp_load": (C.c_int, [vp, vp, u32]),
        "rxg_group_arp_learned": (C.c_int, [vp, u32]),
        "rxg_group_arp_disable": (C.c_int, [vp]),
        "rxg_group_rcv_set": (C.c_int, [vp, i32, u32, u32]),
        "rxg_group_rx_burst": (C.c_int, [vp, C.POINTER(PktView), u32, u32, vp]),
        "rxg_group_rx_replay": (C.c_int, [vp, C.POINTER(HandoffOps), vp, vp, vp, u32, u32]),
        "rxg_group_rx_burst_dev": (C.c_int, [vp, C.POINTER(DevBatch), u32]),
        "rxg_group_sync": (C.c_int, [vp]),
        "rxg_group_counters_rccl_why": (C.c_char_p, [vp]),
        "rxg_group_payload_take": (C.c_int, [vp, i32, u32, u32, C.POINTER(PayloadMsg)]),
        "rxg_group_replaying": (i32, [vp]),
        "rxg_group_counters_reset": (C.c_int, [vp]),
        "rxg_group_counters_read": (C.c_int, [vp, vp]),
        "rxg_group_counters_rccl": (C.c_int, [vp]),
        "rxg_group_last_error": (C.c_char_p, []),
    }
    for name, (res, args) in sig.items():
        if os.path.abspath(path) != _PRODUCT_LIB and not hasattr(lib, name):
            continue  # another build loaded for an A/B (kbench.py, RXG_LIB): its own entry points only
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.rxg_abi_version() != ABI_VERSION:
        raise RxgError(f"librxg ABI version {lib.rxg_abi_version()}, binding expects {ABI_VERSION}")
    _lib = lib
    _loaded_path = path
    return lib


def _check(rc: int, what: str):
    if rc != 0:
        msg = _lib.rxg_last_error().decode(errors="replace") if _lib else ""
        raise RxgError(f"{what} failed ({rc}): {msg}")


def _gcheck(rc: int, what: str):
    if rc != 0:
        msg = _lib.rxg_group_last_error().decode(errors="replace") if _lib else ""
        raise RxgError(f"{what} failed ({rc}): {msg}")


def _ptr(a: np.ndarray) -> int:
    return a.ctypes.data


# ------------------------------------------------------------------------- helpers ---
def pack_arena(frames: list[bytes]) -> tuple[np.ndarray, np.ndarray, np.ndarray]:
    """Pack frames at 64-byte aligned starts (the rxg batch layout).
    Returns (arena u8, off64 u32, len u16)."""
    n = len(frames)
    lens = np.fromiter((len(f) for f in frames), dtype=np.uint32, count=n)
    if n and lens.max() > 0xFFFF:
        raise ValueError("frame longer than 65535 bytes")
    slots = (lens + 63) // 64
    off = np.zeros(n, dtype=np.uint64)
    if n > 1:
        off[1:] = np.cumsum(slots[:-1], dtype=np.uint64)
    total = int(slots.sum()) if n else 0
    arena = np.zeros(max(total * 64, 64), dtype=np.uint8)
    for i, f in enumerate(frames):
        o = int(off[i]) * 64
        arena[o:o + len(f)] = np.frombuffer(f, dtype=np.uint8)
    return arena, off.astype(np.uint32), lens.astype(np.uint16)


def tcb_table(rows) -> tuple[np.ndarray, np.ndarray]:
    """rows: iterable of None (removed slot) or (dport, sport, ipv4_dst_raw, ipv4_src_host,
    state[, identifier]).  Returns (tcbs TCB_DTYPE, live u8)."""
    rows = list(rows)
    t = np.zeros(len(rows), dtype=TCB_DTYPE)
    live = np.zeros(len(rows), dtype=np.uint8)
    for i, r in enumerate(rows):
        if r is None:
            continue
        live[i] = 1
        t[i]["dport"], t[i]["sport"], t[i]["ipv4_dst"], t[i]["ipv4_src"], t[i]["state"] = r[:5]
        t[i]["identifier"] = r[5] if len(r) > 5 else (i % 65535) + 1
    return t, live


def ip_raw(a: int, b: int, c: int, d: int) -> int:
    """An IPv4 address as the reference's u32 load of network-order bytes (x86)."""
    return a | (b << 8) | (c << 16) | (d << 24)


def ip_host(a: int, b: int, c: int, d: int) -> int:
    return (a << 24) | (b << 16) | (c << 8) | d


# -------------------------------------------------------------------------- engine ---
class DevArray:
    """A device allocation owned by an Engine."""

    def __init__(self, eng: "Engine", nbytes: int):
        self.eng, self.nbytes = eng, int(nbytes)
        p = C.c_void_p()
        _check(_lib.rxg_dev_alloc(eng.ctx, max(self.nbytes, 1), C.byref(p)), "rxg_dev_alloc")
        self.ptr = p.value

    def upload(self, a: np.ndarray, stream=None):
        a = np.ascontiguousarray(a)
        if a.nbytes > self.nbytes:
            raise ValueError("upload larger than allocation")
        _check(_lib.rxg_memcpy_h2d(self.eng.ctx, self.ptr, _ptr(a), a.nbytes, stream), "h2d")
        _check(_lib.rxg_stream_sync(self.eng.ctx, stream), "sync")

    def download(self, dtype, count, offset_bytes: int = 0, stream=None) -> np.ndarray:
        out = np.empty(count, dtype=dtype)
        _check(_lib.rxg_memcpy_d2h(self.eng.ctx, _ptr(out), self.ptr + offset_bytes,
                                   out.nbytes, stream), "d2h")
        _check(_lib.rxg_stream_sync(self.eng.ctx, stream), "sync")
        return out

    def free(self):
        if self.ptr:
            _lib.rxg_dev_free(self.eng.ctx, self.ptr)
            self.ptr = None


class PinnedArray:
    """Page-locked host memory (hipHostMalloc) viewed as a numpy uint8 array."""

    def __init__(self, eng: "Engine", nbytes: int):
        self.eng, self.nbytes = eng, int(nbytes)
        p = C.c_void_p()
        _check(_lib.rxg_host_alloc_pinned(eng.ctx, max(self.nbytes, 1), C.byref(p)),
               "rxg_host_alloc_pinned")
        self.ptr = p.value
        self.np = np.ctypeslib.as_array((C.c_uint8 * max(self.nbytes, 1)).from_address(self.ptr))

    def free(self):
        if self.ptr:
            self.np = None
            _lib.rxg_host_free_pinned(self.eng.ctx, self.ptr)
            self.ptr = None


def flow_part_of(frame: bytes, nparts: int) -> int:
    """The RSS queue (0 .. nparts-1) whose context classifies this frame (rxg_flow_part_of)."""
    r = load_library().rxg_flow_part_of(frame, len(frame), nparts)
    if r < 0:
        raise RxgError(f"rxg_flow_part_of failed ({r})")
    return r


def rss_hash(tuple12: bytes) -> int:
    """Toeplitz RSS hash (default Microsoft key) of src ip | dst ip | src port | dst port."""
    assert len(tuple12) == 12
    return load_library().rxg_rss_hash(tuple12)


class Engine:
    """One rxg context on one GPU (include/rxg.h: rxg_init .. rxg_fini)."""

    def __init__(self, device: int = 0, max_batch: int = 0, max_bytes: int = 0,
                 max_blocks: int = 0, zc_bytes: int = 0, flags: int = 0):
        load_library()
        cfg = Config(device, max_batch, max_bytes, flags, max_blocks, zc_bytes)
        ctx = C.c_void_p()
        _check(_lib.rxg_init(C.byref(cfg), C.byref(ctx)), "rxg_init")
        self.ctx = ctx.value
        self.device = device

    @classmethod
    def _member(cls, ctx: int, device: int) -> "Engine":
        """A group member's context, owned by its Group (close() does not free it)."""
        e = cls.__new__(cls)
        e.ctx, e.device, e._borrowed = ctx, device, True
        return e

    def close(self):
        if getattr(self, "ctx", None):
            for d in getattr(self, "_pg_bufs", ()):
                d.free()
            self._pg_bufs = ()
            if not getattr(self, "_borrowed", False):
                _lib.rxg_fini(self.ctx)
            self.ctx = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    @property
    def stream(self) -> int:
        return _lib.rxg_stream(self.ctx)

    def sync(self):
        _check(_lib.rxg_sync(self.ctx), "rxg_sync")

    def stream_register(self, stream: int):
        """rxg_stream_register: a caller stream of a CFG_STREAMS_OUTLIVE_WRITES context."""
        _check(_lib.rxg_stream_register(self.ctx, stream), "rxg_stream_register")

    def stream_retire(self, stream: int):
        """rxg_stream_retire: the stream may be destroyed after this."""
        _check(_lib.rxg_stream_retire(self.ctx, stream), "rxg_stream_retire")

    def host_register(self, a: np.ndarray) -> int:
        """Page-lock and map a host array for zero-copy batches; returns its device alias."""
        d = C.c_void_p()
        _check(_lib.rxg_host_register(self.ctx, _ptr(a), a.nbytes, C.byref(d)), "rxg_host_register")
        return d.value

    def host_unregister(self, a: np.ndarray):
        _check(_lib.rxg_host_unregister(self.ctx, _ptr(a)), "rxg_host_unregister")

    def stream_sync(self, stream):
        _check(_lib.rxg_stream_sync(self.ctx, stream), "rxg_stream_sync")

    def alloc(self, nbytes: int) -> DevArray:
        return DevArray(self, nbytes)

    def pinned(self, nbytes: int) -> PinnedArray:
        return PinnedArray(self, nbytes)

    def h2d(self, dst: int, src: int, nbytes: int, stream=None):
        _check(_lib.rxg_memcpy_h2d(self.ctx, dst, src, nbytes, stream), "rxg_memcpy_h2d")

    def d2h(self, dst: int, src: int, nbytes: int, stream=None):
        _check(_lib.rxg_memcpy_d2h(self.ctx, dst, src, nbytes, stream), "rxg_memcpy_d2h")

    def to_device(self, a: np.ndarray) -> DevArray:
        d = DevArray(self, a.nbytes)
        d.upload(a)
        return d

    # --- TCB mirror
    def tcb_load(self, tcbs: np.ndarray, live: np.ndarray | None = None):
        tcbs = np.ascontiguousarray(tcbs, dtype=TCB_DTYPE)
        lv = None if live is None else np.ascontiguousarray(live, dtype=np.uint8)
        _check(_lib.rxg_tcb_load(self.ctx, _ptr(tcbs), None if lv is None else _ptr(lv),
                                 len(tcbs)), "rxg_tcb_load")

    def tcb_upsert(self, idx: int, dport: int, sport: int, ipv4_dst: int, ipv4_src: int,
                   state: int, identifier: int = 0):
        t = TcbTuple(dport, sport, ipv4_dst, ipv4_src, state, 0, identifier)
        _check(_lib.rxg_tcb_upsert(self.ctx, idx, C.byref(t)), "rxg_tcb_upsert")

    def tcb_remove(self, idx: int):
        _check(_lib.rxg_tcb_remove(self.ctx, idx), "rxg_tcb_remove")

    def tcb_set_state(self, idx: int, state: int):
        _check(_lib.rxg_tcb_set_state(self.ctx, idx, state), "rxg_tcb_set_state")

    def tcb_sync(self):
        _check(_lib.rxg_tcb_sync(self.ctx), "rxg_tcb_sync")

    def tcb_count(self) -> int:
        return _lib.rxg_tcb_count(self.ctx)

    # --- flow-affinity sharding (rxg_flow_partition): this context serves RSS queue `part`
    def flow_partition(self, part: int, nparts: int):
        _check(_lib.rxg_flow_partition(self.ctx, part, nparts), "rxg_flow_partition")

    def tcb_keys(self) -> int:
        return _lib.rxg_tcb_keys(self.ctx)

    # --- writes from other threads (rxg_tcb_post: lock-free, applied at the next burst)
    def tcb_post_upsert(self, idx: int, dport: int, sport: int, ipv4_dst: int, ipv4_src: int,
                        state: int, identifier: int = 0) -> int:
        op = TcbOp(TCB_OP_UPSERT, idx, TcbTuple(dport, sport, ipv4_dst, ipv4_src, state, 0, identifier), 0)
        return _lib.rxg_tcb_post(self.ctx, C.byref(op))

    def tcb_post_remove(self, idx: int) -> int:
        return _lib.rxg_tcb_post(self.ctx, C.byref(TcbOp(TCB_OP_REMOVE, idx)))

    def tcb_post_set_state(self, idx: int, state: int) -> int:
        return _lib.rxg_tcb_post(self.ctx, C.byref(TcbOp(TCB_OP_SET_STATE, idx, TcbTuple(), state)))

    def tcb_drain(self) -> int:
        rc = _lib.rxg_tcb_drain(self.ctx)
        if rc < 0:
            _check(rc, "rxg_tcb_drain")
        return rc

    # --- ARP mirror (ip.c:30-32 learn, arp.c add_mac)
    def arp_load(self, ips):
        a = np.ascontiguousarray(np.asarray(ips, dtype=np.uint32))
        _check(_lib.rxg_arp_load(self.ctx, _ptr(a) if len(a) else None, len(a)), "rxg_arp_load")

    def arp_learned(self, ip: int):
        _check(_lib.rxg_arp_learned(self.ctx, ip & 0xFFFFFFFF), "rxg_arp_learned")

    def arp_count(self) -> int:
        return _lib.rxg_arp_count(self.ctx)

    def arp_disable(self):
        _check(_lib.rxg_arp_disable(self.ctx), "rxg_arp_disable")

    # --- bursts
    def rx_burst_dev(self, frames: int, off64: int, lens: int, n: int, out: int,
                     rec_kind: int = REC16, stream=None):
        b = DevBatch(frames, off64, lens, n, rec_kind, out)
        _check(_lib.rxg_rx_burst_dev(self.ctx, C.byref(b), stream), "rxg_rx_burst_dev")

    def rx_burst_payload_dev(self, frames: int, off64: int, lens: int, n: int, out: int, arena: int,
                             msgs: int, rec_kind: int = REC16, stream=None):
        """rxg_rx_burst_payload_dev: the burst and its payload hand-off in one pass; payload
        lines to `arena` (the frame pool's geometry), one rxg_payload_msg per frame to msgs."""
        b = DevBatch(frames, off64, lens, n, rec_kind, out)
        p = PayloadSlots(arena, msgs)
        _check(_lib.rxg_rx_burst_payload_dev(self.ctx, C.byref(b), C.byref(p), stream), "rxg_rx_burst_payload_dev")

    def rx_burst_strided_payload_dev(self, frames: int, stride64: int, slot0: int, lens: int, n: int, out: int,
                                     arena, msgs: int, rec_kind: int = REC16, stream=None):
        """rxg_rx_burst_strided_payload_dev: one fixed-stride burst and its payload hand-off
        (arena None: by reference)."""
        b = DevStridedBurst(lens, n, slot0, out)
        p = PayloadSlots(arena, msgs)
        _check(_lib.rxg_rx_burst_strided_payload_dev(self.ctx, frames, stride64, C.byref(b), rec_kind, C.byref(p),
                                                     stream), "rxg_rx_burst_strided_payload_dev")

    def rx_bursts_dev(self, frames: int, bursts, rec_kind: int = REC16, stream=None):
        """bursts: [(off64 ptr, len ptr, n, out ptr), ...] of one frame pool, one launch."""
        arr = (DevBurst * max(len(bursts), 1))(*[DevBurst(o, l, n, 0, out) for o, l, n, out in bursts])
        _check(_lib.rxg_rx_bursts_dev(self.ctx, frames, arr, len(bursts), rec_kind, stream),
               "rxg_rx_bursts_dev")

    def rx_bursts_strided_dev(self, frames: int, stride64: int, bursts, rec_kind: int = REC16, stream=None):
        """bursts: [(slot0, len ptr, n, out ptr), ...]: frame i of a burst at 64-byte slot
        slot0 + i * stride64 of the pool (no offset list), one launch."""
        arr = (DevStridedBurst * max(len(bursts), 1))(*[DevStridedBurst(l, n, s0, out) for s0, l, n, out in bursts])
        _check(_lib.rxg_rx_bursts_strided_dev(self.ctx, frames, stride64, arr, len(bursts), rec_kind, stream),
               "rxg_rx_bursts_strided_dev")

    # --- latency mode (rxg_server_*): a persistent kernel serves small bursts
    def server_start(self, rec_kind: int = REC8, blocks: int = 1, max_frames: int = 4096,
                     max_bytes: int = 0, idle_ms: int = 1000, flags: int = 0):
        cfg = ServerConfig(rec_kind, blocks, max_frames, max_bytes, idle_ms, flags)
        _check(_lib.rxg_server_start(self.ctx, C.byref(cfg)), "rxg_server_start")

    def server_placement(self) -> int:
        """SRV_NONE / SRV_HOST (coherent host memory) / SRV_DEVICE (device memory, BAR writes)."""
        return int(_lib.rxg_server_placement(self.ctx))

    def server_stop(self):
        _check(_lib.rxg_server_stop(self.ctx), "rxg_server_stop")

    def server_active(self) -> bool:
        return bool(_lib.rxg_server_active(self.ctx))

    def server_burst_dev(self, frames: int, off64: int, lens: int, n: int, out: int, rec_kind: int = REC8):
        """Synchronous: the records are at `out` on return."""
        b = DevBatch(frames, off64, lens, n, rec_kind, out)
        _check(_lib.rxg_server_burst_dev(self.ctx, C.byref(b)), "rxg_server_burst_dev")

    def tx_cksum_dev(self, frames: int, off64: int, lens: int, n: int, stream=None):
        b = DevTxBatch(frames, off64, lens, n, 0)
        _check(_lib.rxg_tx_cksum_dev(self.ctx, C.byref(b), stream), "rxg_tx_cksum_dev")

    def rx_arena(self, arena: np.ndarray, off64: np.ndarray, lens: np.ndarray,
                 rec_kind: int = REC48) -> np.ndarray:
        """Upload a packed arena, run one burst, return the records (numpy)."""
        n = len(lens)
        dt = rec_dtype(rec_kind)
        if n == 0:
            return np.zeros(0, dtype=dt)
        da, do, dl = self.to_device(arena), self.to_device(off64), self.to_device(lens)
        dout = self.alloc(n * rec_kind)
        try:
            self.rx_burst_dev(da.ptr, do.ptr, dl.ptr, n, dout.ptr, rec_kind)
            self.sync()
            return dout.download(dt, n)
        finally:
            for d in (da, do, dl, dout):
                d.free()

    def tx_arena(self, arena: np.ndarray, off64: np.ndarray, lens: np.ndarray) -> np.ndarray:
        """Run the tx checksum-generate kernel over a packed arena; returns the new arena."""
        n = len(lens)
        if n == 0:
            return arena.copy()
        da, do, dl = self.to_device(arena), self.to_device(off64), self.to_device(lens)
        try:
            self.tx_cksum_dev(da.ptr, do.ptr, dl.ptr, n)
            self.sync()
            return da.download(np.uint8, arena.size)
        finally:
            for d in (da, do, dl):
                d.free()

    def rx_burst(self, frames: list[bytes], rec_kind: int = REC48) -> np.ndarray:
        """rxg_rx_burst over host buffers (DPDK-style views into Python bytes)."""
        n = len(frames)
        bufs = [C.create_string_buffer(f, len(f) + 1) for f in frames]
        views = (PktView * max(n, 1))()
        for i, b in enumerate(bufs):
            views[i] = PktView(C.addressof(b), 0, len(frames[i]), 0)
        dt = rec_dtype(rec_kind)
        out = np.zeros(n, dtype=dt)
        _check(_lib.rxg_rx_burst(self.ctx, views, n, rec_kind, _ptr(out) if n else None),
               "rxg_rx_burst")
        return out

    # --- payload hand-off
    def payload_gather_dev(self, arena: int, arena_cap: int, msgs: int, used: int, stream=None):
        o = PayloadOut(arena, arena_cap, msgs, used)
        _check(_lib.rxg_payload_gather_dev(self.ctx, C.byref(o), stream), "rxg_payload_gather_dev")

    def payload_gather(self, n: int, arena_cap: int):
        """Gather the last burst's payloads; returns (arena bytes, msgs, bytes needed).  The
        device buffers live until the next call (rxg_payload_take reads the descriptors)."""
        for d in getattr(self, "_pg_bufs", ()):
            d.free()
        da, dm, du = self.alloc(max(arena_cap, 16)), self.alloc(max(n, 1) * 16), self.alloc(8)
        self._pg_bufs = (da, dm, du)
        self.payload_gather_dev(da.ptr, arena_cap, dm.ptr, du.ptr)
        self.sync()
        msgs = dm.download(PAYLOAD_MSG_DTYPE, n) if n else np.zeros(0, PAYLOAD_MSG_DTYPE)
        used = int(du.download(np.uint64, 1)[0])
        arena = da.download(np.uint8, min(arena_cap, used)) if arena_cap else np.zeros(0, np.uint8)
        return arena, msgs, used

    def rx_burst_payload(self, frames, rec_kind: int = REC16, arena_fill: int | None = None,
                         by_reference: bool = False):
        """Host frames through rxg_rx_burst_payload_dev (packed, uploaded): returns (records of
        rec_kind,
        payload arena as np.uint8 -- the pool's geometry -- , msgs, (arena, off64, lens) as
        packed).  arena_fill: the payload arena's bytes before the call (None: zeros);
        by_reference: no arena (the messages name the pool, which is then returned).  The
        device buffers live until the next call (the replay reads the batch, rxg_payload_take
        the messages)."""
        for d in getattr(self, "_pf_bufs", ()):
            d.free()
        arena, off, lens = pack_arena(frames)
        n = len(frames)
        da, do, dl = self.to_device(arena), self.to_device(off), self.to_device(lens)
        dr, dm = self.alloc(max(n, 1) * rec_kind), self.alloc(max(n, 1) * 16)
        dp = None
        if not by_reference:
            dp = self.alloc(max(arena.nbytes, 64))
            dp.upload(np.full(max(arena.nbytes, 64), 0 if arena_fill is None else arena_fill, dtype=np.uint8))
        self._pf_bufs = tuple(d for d in (da, do, dl, dr, dm, dp) if d is not None)
        self.rx_burst_payload_dev(da.ptr, do.ptr, dl.ptr, n, dr.ptr, dp.ptr if dp else None, dm.ptr, rec_kind)
        self.sync()
        recs = dr.download(rec_dtype(rec_kind), n)  # as the kernel wrote them (rec8_expand for REC8)
        msgs = dm.download(PAYLOAD_MSG_DTYPE, n) if n else np.zeros(0, PAYLOAD_MSG_DTYPE)
        # by reference the payloads are read from the pool itself (the uploaded batch)
        pay = da.download(np.uint8, arena.nbytes) if by_reference else dp.download(np.uint8, arena.nbytes)
        return recs, pay, msgs, (arena, off, lens)

    def rcv_set(self, idx: int, cur_seq: int, pairs_pending: bool):
        _check(_lib.rxg_rcv_set(self.ctx, idx, cur_seq & 0xFFFFFFFF, int(bool(pairs_pending))),
               "rxg_rcv_set")

    def payload_take(self, idx: int, seq: int, length: int):
        """Inside a replay handler: (True, arena_off) if the gathered payload is the message."""
        m = PayloadMsg()
        rc = _lib.rxg_payload_take(self.ctx, idx, seq & 0xFFFFFFFF, length, C.byref(m))
        _check(min(rc, 0), "rxg_payload_take")
        return rc == 1, int(m.arena_off)

    def replay_stats(self) -> dict:
        out = np.zeros(4, dtype=np.uint64)
        _check(_lib.rxg_replay_stats(self.ctx, _ptr(out)), "rxg_replay_stats")
        return dict(zip(("marked", "host_fixups", "device_fixups", "device_launches"), out.tolist()))

    # --- counters
    def counters_reset(self, stream=None):
        _check(_lib.rxg_counters_reset(self.ctx, stream), "rxg_counters_reset")

    def counters(self) -> np.ndarray:
        out = np.zeros(NCOUNTERS, dtype=np.uint64)
        _check(_lib.rxg_counters_read(self.ctx, _ptr(out)), "rxg_counters_read")
        return out

    def counters_dev_ptr(self) -> int:
        return _lib.rxg_counters_dev(self.ctx)

    # --- synthetic traffic
    def synth(self, n: int, nflows: int, len_a: int = 1500, mix: int = 0,
              seed: int = 0x5EED, dst_ip_host: int = 0xC0A84E02, dport: int = 80,
              with_flows: bool = False, stream=None):
        """Generate n synthetic frames on the device.  Returns a dict of DevArrays."""
        p = SynthParams(seed, n, nflows, dst_ip_host, dport, mix, len_a if mix == 0 else 0, 0)
        nbytes = int(_lib.rxg_synth_arena_bytes(C.byref(p)))
        arena = self.alloc(nbytes)
        off = self.alloc(n * 4)
        lens = self.alloc(n * 2)
        flows = self.alloc(n * 4) if with_flows else None
        used = C.c_uint64()
        _check(_lib.rxg_synth_dev(self.ctx, C.byref(p), arena.ptr, nbytes, off.ptr, lens.ptr,
                                  flows.ptr if flows else None, C.byref(used), stream),
               "rxg_synth_dev")
        return {"arena": arena, "off64": off, "len": lens, "flow": flows, "n": n,
                "arena_bytes": nbytes}

    # --- events
    def event(self):
        e = C.c_void_p()
        _check(_lib.rxg_event_create(self.ctx, C.byref(e)), "rxg_event_create")
        return e.value

    def event_destroy(self, ev):
        _check(_lib.rxg_event_destroy(self.ctx, ev), "rxg_event_destroy")

    def record(self, ev, stream=None):
        _check(_lib.rxg_event_record(self.ctx, ev, stream), "rxg_event_record")

    def elapsed_ms(self, a, b) -> float:
        ms = C.c_float()
        _check(_lib.rxg_event_elapsed_ms(self.ctx, a, b, C.byref(ms)), "rxg_event_elapsed_ms")
        return ms.value


class Group:
    """Several contexts behind one rx loop (include/rxg.h: rxg_group_*).  The mirror calls
    go to every member; rx_burst shards a burst over the members and returns its records in
    packet order; replay() replays the shards in packet order."""

    def __init__(self, devices, max_batch: int = 0, max_bytes: int = 0):
        load_library()
        devs = (C.c_int32 * len(devices))(*devices)
        cfg = Config(0, max_batch, max_bytes, 0, 0, 0)
        g = C.c_void_p()
        _gcheck(_lib.rxg_group_init(devs, len(devices), C.byref(cfg), C.byref(g)), "rxg_group_init")
        self.g = g.value
        self.members = [Engine._member(_lib.rxg_group_member(self.g, i), d) for i, d in enumerate(devices)]

    def close(self):
        if getattr(self, "g", None):
            for m in self.members:
                m.close()
            _lib.rxg_group_fini(self.g)
            self.g = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __len__(self):
        return _lib.rxg_group_size(self.g)

    def tcb_load(self, tcbs: np.ndarray, live: np.ndarray | None = None):
        tcbs = np.ascontiguousarray(tcbs, dtype=TCB_DTYPE)
        lv = None if live is None else np.ascontiguousarray(live, dtype=np.uint8)
        _gcheck(_lib.rxg_group_tcb_load(self.g, _ptr(tcbs), None if lv is None else _ptr(lv), len(tcbs)),
                "rxg_group_tcb_load")

    def tcb_upsert(self, idx: int, dport: int, sport: int, ipv4_dst: int, ipv4_src: int,
                   state: int, identifier: int = 0):
        t = TcbTuple(dport, sport, ipv4_dst, ipv4_src, state, 0, identifier)
        _gcheck(_lib.rxg_group_tcb_upsert(self.g, idx, C.byref(t)), "rxg_group_tcb_upsert")

    def tcb_remove(self, idx: int):
        _gcheck(_lib.rxg_group_tcb_remove(self.g, idx), "rxg_group_tcb_remove")

    def tcb_set_state(self, idx: int, state: int):
        _gcheck(_lib.rxg_group_tcb_set_state(self.g, idx, state), "rxg_group_tcb_set_state")

    def tcb_post_upsert(self, idx: int, dport: int, sport: int, ipv4_dst: int, ipv4_src: int,
                        state: int, identifier: int = 0) -> int:
        op = TcbOp(TCB_OP_UPSERT, idx, TcbTuple(dport, sport, ipv4_dst, ipv4_src, state, 0, identifier), 0)
        return _lib.rxg_group_tcb_post(self.g, C.byref(op))

    def tcb_post_remove(self, idx: int) -> int:
        return _lib.rxg_group_tcb_post(self.g, C.byref(TcbOp(TCB_OP_REMOVE, idx)))

    def tcb_post_set_state(self, idx: int, state: int) -> int:
        return _lib.rxg_group_tcb_post(self.g, C.byref(TcbOp(TCB_OP_SET_STATE, idx, TcbTuple(), state)))

    def tcb_drain(self) -> int:
        rc = _lib.rxg_group_tcb_drain(self.g)
        if rc < 0:
            _gcheck(rc, "rxg_group_tcb_drain")
        return rc

    def arp_load(self, ips):
        a = np.ascontiguousarray(np.asarray(ips, dtype=np.uint32))
        _gcheck(_lib.rxg_group_arp_load(self.g, _ptr(a) if len(a) else None, len(a)), "rxg_group_arp_load")

    def arp_learned(self, ip: int):
        _gcheck(_lib.rxg_group_arp_learned(self.g, ip & 0xFFFFFFFF), "rxg_group_arp_learned")

    def arp_disable(self):
        _gcheck(_lib.rxg_group_arp_disable(self.g), "rxg_group_arp_disable")

    def rcv_set(self, idx: int, cur_seq: int, pairs_pending: bool):
        _gcheck(_lib.rxg_group_rcv_set(self.g, idx, cur_seq & 0xFFFFFFFF, int(bool(pairs_pending))),
                "rxg_group_rcv_set")

    def rx_burst(self, frames: list[bytes], rec_kind: int = REC48) -> np.ndarray:
        n = len(frames)
        bufs = [C.create_string_buffer(f, len(f) + 1) for f in frames]
        views = (PktView * max(n, 1))()
        for i, b in enumerate(bufs):
            views[i] = PktView(C.addressof(b), 0, len(frames[i]), 0)
        dt = rec_dtype(rec_kind)
        out = np.zeros(n, dtype=dt)
        _gcheck(_lib.rxg_group_rx_burst(self.g, views, n, rec_kind, _ptr(out) if n else None),
                "rxg_group_rx_burst")
        return out

    def rx_burst_dev(self, shards, rec_kind: int = REC16):
        """rxg_group_rx_burst_dev: shards[i] = (frames ptr, off64 ptr, len ptr, n, out ptr) in
        memory member i reads, member i's contiguous share of the burst in packet order.
        Asynchronous; sync() waits."""
        arr = (DevBatch * max(len(shards), 1))(*[DevBatch(f, o, l, n, rec_kind, out) for f, o, l, n, out in shards])
        _gcheck(_lib.rxg_group_rx_burst_dev(self.g, arr, len(shards)), "rxg_group_rx_burst_dev")

    def sync(self):
        _gcheck(_lib.rxg_group_sync(self.g), "rxg_group_sync")

    def rx_replay(self, ops, mbufs, frames, recs, n: int, stride: int):
        """rxg_group_rx_replay with ctypes arguments (HandoffOps, void* arrays, record pointer)."""
        _gcheck(_lib.rxg_group_rx_replay(self.g, C.byref(ops), mbufs, frames, recs, n, stride),
                "rxg_group_rx_replay")

    def replaying(self) -> int:
        return _lib.rxg_group_replaying(self.g)

    def payload_take(self, idx: int, seq: int, length: int):
        m = PayloadMsg()
        rc = _lib.rxg_group_payload_take(self.g, idx, seq & 0xFFFFFFFF, length, C.byref(m))
        _gcheck(min(rc, 0), "rxg_group_payload_take")
        return rc == 1, int(m.arena_off)

    def counters_reset(self):
        _gcheck(_lib.rxg_group_counters_reset(self.g), "rxg_group_counters_reset")

    def counters(self) -> np.ndarray:
        out = np.zeros(NCOUNTERS, dtype=np.uint64)
        _gcheck(_lib.rxg_group_counters_read(self.g, _ptr(out)), "rxg_group_counters_read")
        return out

    def counters_rccl(self) -> bool:
        """True when the counter merge is an RCCL all-reduce (members on distinct GPUs)."""
        rc = _lib.rxg_group_counters_rccl(self.g)
        _gcheck(min(rc, 0), "rxg_group_counters_rccl")
        return rc == 1

    def counters_rccl_why(self) -> str:
        """Why the merge runs on the host ('' when it is RCCL)."""
        return _lib.rxg_group_counters_rccl_why(self.g).decode(errors="replace")


def synthetic_tcb_table(nflows: int, dst_raw: int = None, dport: int = 80):
    """TCB table of SURVEY.md §8(d): slot 0 = LISTENING on dport (socket_bind leaves sport 0,
    ipv4_dst network order, socket_interface.c:69-85); slot 1+f = ESTABLISHED child of flow f
    as tcp_listen fills it (tcp_states.c:185-188)."""
    if dst_raw is None:
        dst_raw = ip_raw(192, 168, 78, 2)
    t = np.zeros(nflows + 1, dtype=TCB_DTYPE)
    t[0] = (dport, 0, dst_raw, 0, LISTENING, 0, 1)
    f = np.arange(nflows, dtype=np.uint64)
    t["dport"][1:] = dport
    t["sport"][1:] = (1024 + f % 64511).astype(np.int32)
    t["ipv4_dst"][1:] = dst_raw
    t["ipv4_src"][1:] = ((10 << 24) | (((f >> 16) & 255) << 16) | (((f >> 8) & 255) << 8)
                         | (f & 255)).astype(np.uint32)
    t["state"][1:] = TCP_ESTABLISHED
    t["identifier"][1:] = ((f + 1) % 65535 + 1).astype(np.uint16)
    return t, np.ones(nflows + 1, dtype=np.uint8)
