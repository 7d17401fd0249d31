#!/bin/bash
# r05c: fused payload forms A/B (production form 1 against forms 2 / 3 / 4), then the fused
# and mirror tests.
set -u
O=gpurun_out/r05c; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python3 -u scripts/fusedbench.py --variants ${VARIANTS:-0,101,102,103} --rounds 3 --steps 20 > $O/fused_ab.jsonl 2> $O/fused_ab.err || { echo "STOP fusedbench"; tail -30 $O/fused_ab.err; exit 1; }
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu tests/test_gpu_fused.py tests/test_gpu_mirror.py > $O/pytest.log 2>&1 || { echo "STOP pytest"; tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
echo r05c done
