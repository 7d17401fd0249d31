"""CPU tests of the drop-in boundary: librxg.so loads and exports every entry point that
include/rxg.h declares; the Python mirror's constants and layouts match the header."""
import ctypes as C
import os
import re
import subprocess

import numpy as np
import pytest

import rxg

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "rxg.h")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    inline = set(re.findall(r"static inline [^(]*?\b(rxg_[a-z0-9_]+)\s*\(", src))  # header-only helpers
    return sorted(set(re.findall(r"\b(rxg_[a-z0-9_]+)\s*\(", src)) - inline)


def test_header_declares_the_boundary():
    names = declared_functions()
    for must in ["rxg_init", "rxg_fini", "rxg_rx_burst_dev", "rxg_rx_burst", "rxg_rx_replay",
                 "rxg_tcb_upsert", "rxg_tcb_remove", "rxg_tcb_set_state", "rxg_tx_cksum_dev",
                 "rxg_counters_read", "rxg_counters_dev"]:
        assert must in names


def test_library_exports_every_declared_symbol():
    lib = rxg.load_library()
    missing = [n for n in declared_functions() if not hasattr(lib, n)]
    assert not missing, missing
    out = subprocess.run(["nm", "-D", "--defined-only", rxg.LIB_PATH], capture_output=True,
                         text=True, check=True).stdout
    exported = set(re.findall(r"\bT (rxg_\w+)", out))
    assert set(declared_functions()) <= exported


def test_library_exports_only_the_c_abi():
    """A linker version script (csrc/rxg.map) keeps the C++ internals -- the context helpers
    of csrc/rxg_ctx.h, the rxg:: host functions, the standard-library instantiations -- out
    of the dynamic symbol table: every defined export is an rxg_* entry point."""
    out = subprocess.run(["nm", "-D", "--defined-only", rxg.LIB_PATH], capture_output=True,
                         text=True, check=True).stdout
    names = [line.split()[-1] for line in out.splitlines() if line.strip()]
    assert names and all(n.startswith("rxg_") for n in names), [n for n in names if not n.startswith("rxg_")][:10]


def test_library_has_gfx950_code_object():
    data = open(rxg.LIB_PATH, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in data


def test_abi_version_and_build_info():
    lib = rxg.load_library()
    assert lib.rxg_abi_version() == rxg.ABI_VERSION == 2
    assert b"gfx950" in lib.rxg_build_info()


def test_build_info_names_this_source_tree():
    """rxg_build_info carries the product sources' hash (Makefile SRC_HASH); the library under
    test was built from exactly the sources in this tree, and the hash is computed the same
    way on both sides."""
    prov = rxg.build_provenance()
    assert "src=" + prov["source_hash"] in prov["build"], prov
    assert prov["build_matches_tree"], prov
    assert " rev=" in prov["build"]
    assert prov["lib"] == os.path.abspath(rxg._PRODUCT_LIB)


def _load_in_child(env_extra):
    import sys
    code = ("import sys; sys.path.insert(0, %r); import rxg\n"
            "try:\n    rxg.load_library(); print('LOADED', rxg._loaded_path)\n"
            "except rxg.RxgError as e:\n    print('REFUSED', e)\n") % os.path.join(ROOT, "dpdk-tcpipstack_amd")
    env = {k: v for k, v in os.environ.items() if k not in ("RXG_LIB", "RXG_LIB_OVERRIDE")}
    env.update(env_extra)
    return subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, env=env,
                          timeout=120).stdout


def test_rxg_lib_override_needs_opt_in(tmp_path):
    """RXG_LIB alone never swaps the product library: it is refused
    loudly; with RXG_LIB_OVERRIDE=1 the named build (here a copy of the product one) is
    loaded; unset, the product one."""
    import shutil
    other = str(tmp_path / "librxg_other.so")
    shutil.copy(rxg.LIB_PATH, other)
    out = _load_in_child({"RXG_LIB": other})
    assert out.startswith("REFUSED") and "RXG_LIB_OVERRIDE=1" in out, out
    out = _load_in_child({"RXG_LIB": other, "RXG_LIB_OVERRIDE": "1"})
    assert out.strip() == "LOADED " + other, out
    out = _load_in_child({})
    assert out.strip() == "LOADED " + rxg._PRODUCT_LIB, out


def test_struct_layouts_match_header():
    hdr = open(HEADER).read()
    src = r'''
#include <stdio.h>
#include <stddef.h>
#include "rxg.h"
int main(void) {
  printf("%zu %zu %zu %zu %zu %zu %zu %d %zu\n", sizeof(rxg_rec16), sizeof(rxg_rec48),
         sizeof(rxg_tcb_tuple), sizeof(rxg_dev_batch), sizeof(rxg_pkt_view),
         sizeof(rxg_synth_params), offsetof(rxg_rec48, src_mac), RXG_NCOUNTERS, sizeof(rxg_tcb_op));
  return 0;
}'''
    tmp = os.path.join(ROOT, "build_abi_probe")
    os.makedirs(tmp, exist_ok=True)
    with open(os.path.join(tmp, "p.c"), "w") as fh:
        fh.write(src)
    subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), os.path.join(tmp, "p.c"), "-o",
                    os.path.join(tmp, "p")], check=True)
    got = subprocess.run([os.path.join(tmp, "p")], capture_output=True, text=True).stdout.split()
    assert [int(x) for x in got] == [16, 48, 20, C.sizeof(rxg.DevBatch), C.sizeof(rxg.PktView),
                                     C.sizeof(rxg.SynthParams), 41, rxg.NCOUNTERS, C.sizeof(rxg.TcbOp)]
    assert rxg.REC48_DTYPE.fields["src_mac"][1] == 41
    assert "RXG_NCOUNTERS" in hdr


def test_python_constants_match_header():
    hdr = open(HEADER).read()
    enum = re.search(r"enum rxg_counter \{(.*?)\};", hdr, re.S).group(1)
    names = [m.lower()[6:] for m in re.findall(r"\b(RXG_C_[A-Z0-9_]+)", enum)]
    assert names == rxg.COUNTERS
    for name, val in [("RXG_V_DISPATCH", 0), ("RXG_V_RST_NOPCB", 1), ("RXG_V_RST_LISTEN_NONSYN", 2),
                      ("RXG_V_DROP_NONTCP", 3), ("RXG_V_ARP", 4), ("RXG_V_DROP_L2", 5)]:
        assert re.search(rf"{name} = {val}\b", hdr)


def test_no_gpu_fails_loudly():
    """Without a GPU the engine refuses to run (no CPU fallback)."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(rxg.RxgError, match="rxg_init"):
        rxg.Engine(0)


def test_group_and_null_arguments_fail_loudly():
    """Group init without a GPU, and NULL arguments everywhere, return negative errno with a
    message; nothing crashes and nothing falls back to the CPU."""
    import ctypes as C
    import torch
    lib = rxg.load_library()
    g = C.c_void_p()
    if not torch.cuda.is_available():
        devs = (C.c_int32 * 2)(0, 0)
        assert lib.rxg_group_init(devs, 2, None, C.byref(g)) < 0
        assert b"rxg_init" in lib.rxg_last_error() or lib.rxg_group_last_error()
    assert lib.rxg_group_init(None, 0, None, C.byref(g)) == -22
    assert b"bad argument" in lib.rxg_group_last_error()
    assert lib.rxg_group_size(None) == 0 and lib.rxg_group_member(None, 0) is None
    assert lib.rxg_group_tcb_post(None, None) == -22
    assert lib.rxg_group_rx_burst(None, None, 0, 16, None) == -22
    assert lib.rxg_group_replaying(None) == -22
    d = C.c_void_p()
    assert lib.rxg_host_register(None, None, 0, C.byref(d)) == -22
    assert lib.rxg_tcb_post(None, None) == -22
    assert lib.rxg_rx_burst(None, None, 0, 16, None) == -22
    # latency mode (rxg_server_*): no context
    cfg = rxg.ServerConfig(rxg.REC8, 1, 32, 0, 0, 0)
    assert lib.rxg_server_start(None, C.byref(cfg)) == -22
    assert lib.rxg_server_stop(None) == -22
    assert lib.rxg_server_active(None) == 0
    assert lib.rxg_server_placement(None) == 0
    assert lib.rxg_server_burst_dev(None, None) == -22


def test_server_config_layout_matches_header():
    import ctypes as C
    src = r'''
#include <stdio.h>
#include <stddef.h>
#include "rxg.h"
int main(void) {
  printf("%zu %zu %zu %zu %u %u %d %d %d\n", sizeof(rxg_server_config), offsetof(rxg_server_config, max_bytes),
         offsetof(rxg_server_config, idle_ms), offsetof(rxg_server_config, flags), RXG_SRV_HOST_STAGING,
         RXG_SRV_HOST_MAILBOX, RXG_SRV_NONE, RXG_SRV_HOST, RXG_SRV_DEVICE);
  return 0;
}'''
    tmp = os.path.join(ROOT, "build_abi_probe")
    os.makedirs(tmp, exist_ok=True)
    with open(os.path.join(tmp, "srv.c"), "w") as fh:
        fh.write(src)
    subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), os.path.join(tmp, "srv.c"), "-o",
                    os.path.join(tmp, "srv")], check=True)
    got = subprocess.run([os.path.join(tmp, "srv")], capture_output=True, text=True, check=True).stdout.split()
    assert [int(x) for x in got] == [C.sizeof(rxg.ServerConfig), rxg.ServerConfig.max_bytes.offset,
                                     rxg.ServerConfig.idle_ms.offset, rxg.ServerConfig.flags.offset,
                                     rxg.SRV_HOST_STAGING, rxg.SRV_HOST_MAILBOX, rxg.SRV_NONE, rxg.SRV_HOST,
                                     rxg.SRV_DEVICE]


def test_product_does_not_link_the_oracle():
    out = subprocess.run(["readelf", "-d", rxg.LIB_PATH], capture_output=True, text=True,
                         check=True).stdout
    assert "oracle" not in out
    syms = subprocess.run(["nm", "-D", rxg.LIB_PATH], capture_output=True, text=True).stdout
    assert "orc_" not in syms


def test_product_does_not_need_rccl_at_load():
    """RCCL serves only the group's counter merge over distinct GPUs; it is
    dlopen'ed there, so single-GPU users and the plain-C rx loop load librxg.so without it."""
    out = subprocess.run(["readelf", "-d", rxg.LIB_PATH], capture_output=True, text=True,
                         check=True).stdout
    needed = [line for line in out.splitlines() if "(NEEDED)" in line]
    assert needed and not any("rccl" in line for line in needed), needed


def test_pack_arena_layout():
    frames = [b"a" * 10, b"b" * 64, b"c" * 65, b""]
    arena, off, lens = rxg.pack_arena(frames)
    assert off.tolist() == [0, 1, 2, 4] and lens.tolist() == [10, 64, 65, 0]
    assert arena.size == 4 * 64 and bytes(arena[128:193]) == b"c" * 65


# the environment switches rounds 1-5's experiment build read (retired in round 6)
EXPERIMENT_SWITCHES = [b"RXG_VARIANT", b"RXG_NOCOUNT", b"RXG_PG_VARIANT", b"RXG_MAX_BLOCKS", b"RXG_ZC_BYTES",
                       b"RXG_MIRROR_REBUILD", b"RXG_REPLAY_COARSE", b"RXG_LAUNCH_PATCHES", b"RXG_MIRROR_LOAD_PCT"]


def _kernel_instantiations(path):
    """(MODE, DESC, MULTI, DEEP, PAY) of every rx_kernel in the library's gfx950 code object
    (csrc/rxg_rx.h: rx_kernel<MODE, DESC, MULTI, DEEP, PAY>)."""
    data = open(path, "rb").read()
    return {tuple(int(x) for x in m) for m in
            re.findall(rb"rx_kernelILi(\d+)ELi(\d+)ELb(\d)ELb(\d)ELi(\d)EEEv", data)}


# The product kernels: round 3's set (every record kind single / multi-burst, the two-deep
# REC8 / REC16 forms, tx, the REC16 re-classification through a selection list), the
# fixed-stride forms (DESC 2, rxg_rx_bursts_strided_dev), and round 5's fused payload
# hand-off (rxg_rx_burst_payload_dev: one burst, every record kind, list or stride; PAY 1 with
# the payload copied, PAY 2 by reference).
PRODUCT_KERNELS = ({(m, d, mu, dp, 0) for m in (8, 16) for d in (0, 2) for mu in (0, 1) for dp in (0, 1)}
                   | {(48, d, mu, 0, 0) for d in (0, 2) for mu in (0, 1)}
                   | {(0, 0, 0, 0, 0), (16, 1, 0, 0, 0)}
                   | {(m, d, 0, 0, p) for m in (8, 16, 48) for d in (0, 2) for p in (1, 2)})


def test_product_library_has_no_experiment_switches():
    """librxg.so reads no environment variable that changes what a burst computes and holds
    only the production kernels, exactly PRODUCT_KERNELS (no ablation
    template parameter is left in rx_kernel / rx_server; their round-2..5 measurements are in
    HISTORY.md)."""
    data = open(rxg.LIB_PATH, "rb").read()
    for sw in EXPERIMENT_SWITCHES:
        assert sw not in data, sw
    inst = _kernel_instantiations(rxg.LIB_PATH)
    assert inst == PRODUCT_KERNELS, sorted(inst ^ PRODUCT_KERNELS)
    servers = set(re.findall(rb"rx_serverILi(\d+)EEEv", data))
    assert servers == {b"8", b"16", b"48"}, servers
    assert not re.findall(rb"rx_serverILi\d+ELi", data)  # no second (stamp / ablation) parameter
    assert re.findall(rb"pg_gather", data)


def test_no_experiment_build_remains():
    """the experiment library (librxg_exp.so, its ablation kernels and
    environment switches) is retired.  build() compiles only what a test, smoke or the bench
    loads: the product library, its example programs and the oracle."""
    pkg = os.path.join(ROOT, "dpdk-tcpipstack_amd")
    mk = open(os.path.join(pkg, "Makefile")).read()
    assert "experiments" not in mk and "RXG_EXPERIMENTS" not in mk and "exp-" not in mk
    assert not os.path.exists(os.path.join(pkg, "csrc", "rxg_kernels_exp.hip"))
    ge = open(os.path.join(ROOT, "__graft_entry__.py")).read()
    assert '"experiments"' not in ge


def test_kernel_source_has_no_experiment_branches():
    """no product source keeps experiment
    scaffolding: no RXG_EXPERIMENTS blocks, no STRIP / ablation / stamp bits, and rx_body
    takes at most 6 template parameters."""
    csrc = os.path.join(ROOT, "dpdk-tcpipstack_amd", "csrc")
    for f in sorted(os.listdir(csrc)):
        if not f.endswith((".h", ".hip", ".cpp")):
            continue
        src = open(os.path.join(csrc, f)).read()
        for word in ("RXG_EXPERIMENTS", "STRIP", "ABL", "SRVX", "kAbl", "abl_stamp", "getenv(\"RXG_"):
            assert word not in src, (f, word)
    body = open(os.path.join(csrc, "rxg_rx.h")).read()
    m = re.search(r"template <([^>]*)>\s*__device__ __forceinline__ void rx_body\(", body)
    assert m and len(m.group(1).split(",")) <= 6, m and m.group(1)


def test_handoff_ops_layout_matches_header():
    """rxg_handoff_ops grew the reference's rx counters (tcp_in.c:18-19) and a flags word."""
    src = r'''
#include <stdio.h>
#include <stddef.h>
#include "rxg.h"
int main(void) {
  printf("%zu %zu %zu %zu %zu %zu\n", sizeof(rxg_handoff_ops), offsetof(rxg_handoff_ops, tcpnopcb),
         offsetof(rxg_handoff_ops, tcpchecksumerror), offsetof(rxg_handoff_ops, flags),
         sizeof(rxg_config), offsetof(rxg_config, zc_bytes));
  return 0;
}'''
    tmp = os.path.join(ROOT, "build_abi_probe")
    os.makedirs(tmp, exist_ok=True)
    with open(os.path.join(tmp, "h.c"), "w") as fh:
        fh.write(src)
    subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), os.path.join(tmp, "h.c"), "-o",
                    os.path.join(tmp, "h")], check=True)
    got = [int(x) for x in subprocess.run([os.path.join(tmp, "h")], capture_output=True, text=True).stdout.split()]
    H = rxg.HandoffOps
    assert got == [C.sizeof(H), H.tcpnopcb.offset, H.tcpchecksumerror.offset, H.flags.offset,
                   C.sizeof(rxg.Config), rxg.Config.zc_bytes.offset]


def test_rec8_pack_and_expand_match_header(tmp_path):
    """rxg_rec8 (rxg.h): the Python packer (the kernel's packing) and rxg_rec8_expand round
    trip every record of the oracle's parity set; the checksums come back as 0 / 0xFFFF."""
    import oracle
    import pktgen
    rows, frames = pktgen.parity_set(seed=31, n=3000)
    tcb, live = pktgen.table_arrays(rows)
    exp, _ = oracle.rx_batch(*pktgen.pack_arena(frames), tcb, live)
    r16 = exp["c"].copy()
    r8 = rxg.rec8_pack(r16)
    src = r'''
#include <stdio.h>
#include <stdlib.h>
#include "rxg.h"
int main(int argc, char **argv) {
  FILE *f = fopen(argv[1], "rb"), *o = fopen(argv[2], "wb");
  rxg_rec8 r; rxg_rec16 x;
  while (fread(&r, sizeof r, 1, f) == 1) { rxg_rec8_expand(&r, &x); fwrite(&x, sizeof x, 1, o); }
  fclose(f); fclose(o); return 0;
}'''
    (tmp_path / "e.c").write_text(src)
    subprocess.run(["gcc", "-Wall", "-Werror", "-I", os.path.join(ROOT, "include"), str(tmp_path / "e.c"),
                    "-o", str(tmp_path / "e")], check=True)
    r8.tofile(tmp_path / "in.bin")
    subprocess.run([str(tmp_path / "e"), str(tmp_path / "in.bin"), str(tmp_path / "out.bin")], check=True)
    c_exp = np.fromfile(tmp_path / "out.bin", dtype=rxg.REC16_DTYPE)
    py_exp = rxg.rec8_expand(r8)
    assert c_exp.tobytes() == py_exp.tobytes()
    # everything but the checksum values survives; the checksums as their zero-ness
    for f in ["tcb_idx", "verdict", "state", "tcp_flags", "flags", "datalen"]:
        assert (py_exp[f] == r16[f]).all(), f
    assert ((py_exp["ip_cksum"] == 0) == (r16["ip_cksum"] == 0)).all()
    assert ((py_exp["tcp_cksum"] == 0) == (r16["tcp_cksum"] == 0)).all()
    assert (r16["ip_cksum"] != 0).any() and (r16["tcp_cksum"] != 0).any()
    assert (r16["tcb_idx"] < 0).any() and (r16["state"] == rxg.STATE_NONE).any() and (r16["datalen"] < 0).any()
