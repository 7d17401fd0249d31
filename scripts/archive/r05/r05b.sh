#!/bin/bash
# r05b: the fused rx + payload hand-off on the GPU: its parity tests, the payload / server
# suites it touches, then the bench's fused leg and a rocprof profile of it.
set -u
O=gpurun_out/r05b; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu tests/test_gpu_fused.py tests/test_gpu_payload.py tests/test_gpu_server.py tests/test_gpu_parity.py > $O/pytest.log 2>&1 || { echo "STOP pytest"; tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
timeout -k 10 400 python3 -u bench.py --steps 20 --warmup 5 --no-cpu > $O/bench.json 2> $O/bench.err || { echo "STOP bench"; tail -30 $O/bench.err; exit 1; }
REC=8 bash scripts/gpu_prof.sh r05b pf3 || exit 1
echo r05b done
