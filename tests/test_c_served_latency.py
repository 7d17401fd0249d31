"""examples/served_latency.c (the reference's call site, bursts of MAX_PKT_BURST = 32 at
main.c:116, timed in C through the latency-mode server and the launched path): it builds with
the library's Makefile, refuses bad arguments, and on the GPU prints one JSON line whose served
and launched timings are positive and ordered (p10 <= median <= p90)."""
import json
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "dpdk-tcpipstack_amd")
EXE = os.path.join(PKG, "build", "served_latency")


def _exe():
    if not os.path.exists(EXE):
        subprocess.run(["make", "-s", "-C", PKG, "build/served_latency"], check=True)
    return EXE


def test_builds_and_refuses_bad_arguments():
    exe = _exe()
    assert subprocess.run([exe], capture_output=True).returncode == 2
    assert subprocess.run([exe, "40", "32", "10"], capture_output=True).returncode == 2  # frame < 54 bytes


@pytest.mark.gpu
@pytest.mark.parametrize("args", [["64", "32", "200"], ["1500", "32", "200", "100"]])
def test_served_latency_line(args):
    r = subprocess.run([_exe()] + args, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    d = json.loads(r.stdout.strip().splitlines()[-1])
    assert d["frame_bytes"] == int(args[0]) and d["burst"] == int(args[1])
    for k in ("served_us", "launched_us"):
        assert 0 < d[k]["p10"] <= d[k]["median"] <= d[k]["p90"]
