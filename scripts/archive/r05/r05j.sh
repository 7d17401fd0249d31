#!/bin/bash
# r05j: the tree after the fused kernel's pruning -- every GPU test, smoke, the bench, and the
# fused kernel's rocprof passes (C3 and C4).
set -u
O=gpurun_out/r05j; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu tests/ > $O/pytest.log 2>&1 || { echo "STOP pytest"; tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "STOP smoke"; tail -20 $O/smoke.log; exit 1; }
cat $O/smoke.log
timeout -k 10 400 python3 -u bench.py > $O/bench.json 2> $O/bench.err || { echo "STOP bench"; tail -30 $O/bench.err; exit 1; }
REC=8 bash scripts/gpu_prof.sh r05j pf3 pf4 || exit 1
echo r05j done
