#!/bin/bash
# r05q: the by-reference fused form as its own kernels (PAY = kPayRef: no payload stores or
# line-end loads compiled in) on the record kind's occupancy grid; the copy form beside it.
set -u
O=gpurun_out/r05q; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu tests/test_gpu_fused.py tests/test_abi.py > $O/pytest.log 2>&1 || { echo "STOP pytest"; tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 400 python3 -u scripts/fusedbench.py --by-ref --rounds 3 --steps 20 > $O/byref.jsonl 2> $O/byref.err || { echo "STOP fusedbench by-ref"; tail -30 $O/byref.err; exit 1; }
timeout -k 10 400 python3 -u scripts/fusedbench.py --rounds 3 --steps 20 > $O/copy.jsonl 2> $O/copy.err || { echo "STOP fusedbench copy"; tail -30 $O/copy.err; exit 1; }
timeout -k 10 400 python3 -u bench.py > $O/bench.json 2> $O/bench.err || { echo "STOP bench"; tail -30 $O/bench.err; exit 1; }
echo r05q done
