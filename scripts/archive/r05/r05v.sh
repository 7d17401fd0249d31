#!/bin/bash
# r05v: the by-reference form with 8-byte messages staged in a ring of 12 (REC8) / 8 (REC16)
# slots (50 KB per workgroup: 13 slots measured 2 per CU): the fused tests, timings at the record grid and
# at 2 per CU, then profiled (kernel trace, FETCH_SIZE, WRITE_SIZE).
set -u
O=gpurun_out/r05v; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu tests/test_gpu_fused.py > $O/pytest.log 2>&1 || { echo "STOP pytest"; tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 400 python3 -u scripts/fusedbench.py --by-ref --variants 0,0@512 --rounds 3 --steps 20 > $O/byref.jsonl 2> $O/byref.err || { echo "STOP fusedbench by-ref"; tail -30 $O/byref.err; exit 1; }
REC=8 bash scripts/gpu_prof.sh r05v pr3 || exit 1
echo r05v done
