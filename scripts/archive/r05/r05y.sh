#!/bin/bash
# r05y: the copy form's all-small stores moved after the step's loads (probe, next frames,
# descriptors): fused tests, then the copy form's timings.
set -u
O=gpurun_out/r05y; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu tests/test_gpu_fused.py tests/test_gpu_kernel_paths.py > $O/pytest.log 2>&1 || { echo "STOP pytest"; tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 400 python3 -u scripts/fusedbench.py --rounds 3 --steps 20 > $O/copy.jsonl 2> $O/copy.err || { echo "STOP fusedbench copy"; tail -30 $O/copy.err; exit 1; }
echo r05y done
