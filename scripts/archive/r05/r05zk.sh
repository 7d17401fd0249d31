#!/bin/bash
# r05zk: the opt-in soaks on the shipped tree, 180 s each (launched shapes, served bursts,
# fused forms), bit-exact against the oracle.
set -u
O=gpurun_out/r05zk; mkdir -p $O
export TMPDIR=/tmp
RXG_SOAK=180 timeout -k 10 700 python3 -u -m pytest -x -v -s --timeout 600 --timeout-method thread -m gpu tests/test_gpu_soak.py 2>&1 | tee $O/pytest.log | grep -E --line-buffered "soak|passed|failed|Error" || true
grep -q " 3 passed" $O/pytest.log || { echo "STOP soak"; tail -30 $O/pytest.log; exit 1; }
echo r05zk done
