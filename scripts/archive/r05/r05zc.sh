#!/bin/bash
# r05zc: the fused hand-off soak (opt-in) for 150 s: random batches, grids, record kinds,
# copy and by-reference forms, bit-exact against the oracle.
set -u
O=gpurun_out/r05zc; mkdir -p $O
export TMPDIR=/tmp
RXG_SOAK=150 timeout -k 10 400 python3 -u -m pytest -x -v -s --timeout 380 --timeout-method thread -m gpu tests/test_gpu_soak.py -k fused > $O/pytest.log 2>&1 || { echo "STOP soak"; tail -40 $O/pytest.log; exit 1; }
grep -E "fused soak|passed|failed" $O/pytest.log | tail -4
echo r05zc done
