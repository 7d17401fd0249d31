#!/bin/bash
# r05k: the strided and by-reference fused forms: tests, then the bench.
set -u
O=gpurun_out/r05k; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu tests/test_gpu_fused.py tests/test_gpu_payload.py > $O/pytest.log 2>&1 || { echo "STOP pytest"; tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
timeout -k 10 400 python3 -u bench.py --steps 20 --warmup 5 --no-cpu > $O/bench.json 2> $O/bench.err || { echo "STOP bench"; tail -30 $O/bench.err; exit 1; }
echo r05k done
