#!/bin/bash
# Deferred header derivation (RAW): GPU parity tests, then A/B against the round-2 form (variant 46).
set -u
O=gpurun_out/raw; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernel_paths.py tests/test_gpu_parity.py tests/test_gpu_fullsize.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; echo STOP tests; exit 1; }
tail -1 $O/pytest.log
TAG=raw VARIANTS=0:0,46:0,0:0:x,46:0:x WLS=c4,c3,c2,u576,u1500 bash scripts/gpu_ab.sh
