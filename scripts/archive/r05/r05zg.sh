#!/bin/bash
# r05zg: the opt-in soaks (launched shapes, served bursts, fused forms), 60 s each, on the
# tree whose burst kernels carry the mirror's patch lists.
set -u
O=gpurun_out/r05zg; mkdir -p $O
export TMPDIR=/tmp
RXG_SOAK=60 timeout -k 10 400 python3 -u -m pytest -x -v -s --timeout 300 --timeout-method thread -m gpu tests/test_gpu_soak.py > $O/pytest.log 2>&1 || { echo "STOP soak"; tail -40 $O/pytest.log; exit 1; }
grep -E "soak: .*bit-exact|passed|failed" $O/pytest.log | tail -5
echo r05zg done
