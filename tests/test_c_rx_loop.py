"""The reference's rx loop patched per INTEGRATION.md, in plain C (dpdk-tcpipstack_amd/
examples/rx_loop.c, built by the library's Makefile): C handlers shaped like tcp_states.c's
behind rxg_rx_burst + rxg_rx_replay, mirroring their tcbs[] writes with rxg_tcb_*.  On the
GPU its per-packet outcome and final table equal the sequential reference loop
(tests/test_gpu_replay.py) at burst sizes 1, 32 (MAX_PKT_BURST, main.c:116) and 256; on CPU
it must build, link and fail loudly without a GPU."""
import os
import struct
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "dpdk-tcpipstack_amd")
EXE = os.path.join(PKG, "build", "rx_loop")
ROW = struct.Struct("<iiIIBBH")
OUT = np.dtype([("kind", "u1"), ("state", "u1"), ("pad", "<u2"), ("tcb_idx", "<i4")])


def _exe():
    if not os.path.exists(EXE):
        subprocess.run(["make", "-s", "-C", PKG, "build/rx_loop"], check=True)
    return EXE


def _write_input(path, rows, frames):
    with open(path, "wb") as fh:
        fh.write(struct.pack("<I", len(rows)))
        for r in rows:
            fh.write(ROW.pack(0, 0, 0, 0, 0, 0, 0) if r is None else
                     ROW.pack(r[0], r[1], r[2] & 0xFFFFFFFF, r[3] & 0xFFFFFFFF, r[4], 1, 0))
        fh.write(struct.pack("<I", len(frames)))
        for f in frames:
            fh.write(struct.pack("<H", len(f)) + f)


def _read_output(path, n, with_globals=False):
    data = open(path, "rb").read()
    out = np.frombuffer(data[: n * OUT.itemsize], dtype=OUT)
    (ntcb,) = struct.unpack_from("<I", data, n * OUT.itemsize)
    rows = []
    for i in range(ntcb):
        d, s, dst, src, st, live, _ = ROW.unpack_from(data, n * OUT.itemsize + 4 + i * ROW.size)
        rows.append((d, s, dst, src, st) if live else None)
    if with_globals:  # the reference's rx globals tcpnopcb, tcpchecksumerror (tcp_in.c:18-19)
        g = struct.unpack_from("<ii", data, n * OUT.itemsize + 4 + ntcb * ROW.size)
        return out, rows, {"tcpnopcb": g[0], "tcpchecksumerror": g[1]}
    return out, rows


def test_c_loop_builds_and_fails_loudly_without_gpu(tmp_path):
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present: the GPU test covers the loop")
    inp = tmp_path / "in.bin"
    _write_input(inp, [(80, 0, 0x024EA8C0, 0, 1)], [bytes(60)])
    r = subprocess.run([_exe(), str(inp), str(tmp_path / "out.bin"), "32"], capture_output=True, text=True)
    assert r.returncode == 3 and "rxg_init" in r.stderr, (r.returncode, r.stderr)


@pytest.mark.gpu
@pytest.mark.parametrize("burst,server", [(1, False), (32, False), (256, False), (1, True), (32, True), (256, True)])
def test_c_loop_equals_sequential_reference(tmp_path, burst, server):
    """server: the same loop in latency mode (rxg_server_start, RX_LOOP_SERVER=1)."""
    from test_gpu_replay import scenario, sequential_reference
    import rxg
    rows, frames = scenario(7, n=600 if burst == 1 else 1500)
    exp, _, erows = sequential_reference(rows, frames)
    inp, outp = tmp_path / "in.bin", tmp_path / "out.bin"
    _write_input(inp, rows, frames)
    env = dict(os.environ, RX_LOOP_SERVER="1" if server else "0")
    r = subprocess.run([_exe(), str(inp), str(outp), str(burst)], capture_output=True, text=True, timeout=300,
                       env=env)
    assert r.returncode == 0, r.stderr
    out, got_rows = _read_output(outp, len(frames))
    for i, (v, idx, st) in enumerate(exp):
        if v == rxg.V_DISPATCH:
            assert (out["kind"][i], out["tcb_idx"][i], out["state"][i]) == (3, idx, st), (i, out[i], exp[i])
        elif v in (rxg.V_RST_NOPCB, rxg.V_RST_LISTEN_NONSYN):
            assert out["kind"][i] == 2, (i, out[i], exp[i])
        else:
            assert out["kind"][i] == 1, (i, out[i], exp[i])
    assert [None if x is None else (x[0], x[1], x[2] & 0xFFFFFFFF, x[3] & 0xFFFFFFFF, x[4]) for x in erows] == \
        [None if x is None else tuple(x) for x in got_rows]


@pytest.mark.gpu
@pytest.mark.parametrize("verify", [False, True])
def test_c_loop_reference_rx_counters(tmp_path, verify):
    """tcpnopcb / tcpchecksumerror (tcp_in.c:18-19, extern in tcp_in.h:7,11) stay linkable
    and correct behind the replaced loop: the C program hands their addresses to the replay
    (rxg_handoff_ops), which bumps them in packet order exactly where tcp_in does -- with
    the reference's `if(0)` (verify off) and with the check compiled in (verify on: bad
    TCP checksums freed before findtcb, no reset, no hand-off)."""
    from test_gpu_replay import scenario, sequential_reference
    import rxg
    rows, frames = scenario(11, n=1500, corrupt=0.08, closed=0.1)
    g_exp = {}
    exp, _, erows = sequential_reference(rows, frames, verify=verify, globals_out=g_exp)
    assert g_exp["tcpnopcb"] > 0 and (g_exp["tcpchecksumerror"] > 0) == verify
    inp, outp = tmp_path / "in.bin", tmp_path / "out.bin"
    _write_input(inp, rows, frames)
    args = [_exe(), str(inp), str(outp), "32"] + (["verify"] if verify else [])
    r = subprocess.run(args, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    out, got_rows, g_got = _read_output(outp, len(frames), with_globals=True)
    assert g_got == g_exp
    for i, (v, idx, st) in enumerate(exp):
        if v == rxg.V_DISPATCH:
            assert (out["kind"][i], out["tcb_idx"][i], out["state"][i]) == (3, idx, st), (i, out[i], exp[i])
        elif v in (rxg.V_RST_NOPCB, rxg.V_RST_LISTEN_NONSYN):
            assert out["kind"][i] == 2, (i, out[i], exp[i])
        else:
            assert out["kind"][i] == 1, (i, out[i], exp[i])
    assert [None if x is None else (x[0], x[1], x[2] & 0xFFFFFFFF, x[3] & 0xFFFFFFFF, x[4]) for x in erows] == \
        [None if x is None else tuple(x) for x in got_rows]
