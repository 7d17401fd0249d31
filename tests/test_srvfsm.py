"""CPU: the latency-mode server's host state machine (dpdk-tcpipstack_amd/csrc/rxg_srvfsm.h,
VERDICT r3 item 7).  tests/srvfsm_check.cpp drives it against a scripted
device: after a request misses its time limit the server is Failed, and until its kernel has
exited every call returns -EIO within exit_timeout (no unbounded stream synchronisation, no
post that would cancel the stop); once it exits the next call relaunches and is served.
Built plain and under ASan/UBSan."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "dpdk-tcpipstack_amd", "csrc")


@pytest.mark.parametrize("san", [[], ["-fsanitize=address,undefined", "-fno-sanitize-recover=all"]])
def test_server_state_machine(tmp_path, san):
    exe = tmp_path / "srvfsm_check"
    subprocess.run(["g++", "-O1", "-g", "-std=c++17", "-Wall", "-Wextra", "-Werror", *san, "-I", CSRC,
                    os.path.join(ROOT, "tests", "srvfsm_check.cpp"), "-o", str(exe)], check=True)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:halt_on_error=1")
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode == 0 and "srvfsm ok" in r.stdout, r.stdout + r.stderr
