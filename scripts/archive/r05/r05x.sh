#!/bin/bash
# r05x: new parity tests of the fused forms -- many slices per wave on 1- and 3-workgroup
# grids (the by-reference ring flushing mid-stream) and the by-reference form at full C3 / C4.
set -u
O=gpurun_out/r05x; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu tests/test_gpu_kernel_paths.py tests/test_gpu_fused.py > $O/pytest.log 2>&1 || { echo "STOP pytest"; tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
echo r05x done
