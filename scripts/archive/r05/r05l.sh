#!/bin/bash
# r05l: fused messages staged in the LDS ring: tests, the fused forms' times, the bench.
set -u
O=gpurun_out/r05l; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu tests/test_gpu_fused.py tests/test_gpu_payload.py > $O/pytest.log 2>&1 || { echo "STOP pytest"; tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 python3 -u scripts/fusedbench.py --variants 0 --workloads c3,c4,c2 --rounds 3 --steps 20 > $O/fused.jsonl 2> $O/fused.err || { echo "STOP fusedbench"; tail -30 $O/fused.err; exit 1; }
timeout -k 10 400 python3 -u bench.py --steps 20 --warmup 5 --no-cpu > $O/bench.json 2> $O/bench.err || { echo "STOP bench"; tail -30 $O/bench.err; exit 1; }
echo r05l done
