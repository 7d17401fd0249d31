#!/bin/bash
# Final kernel of the round: GPU tests, rocprofv3 kernel stats + FETCH/WRITE PMC passes
# (C3, C4, C2, C2 multi-burst) and the bench line.  TAG names the gpurun_out directory.
set -u
export TMPDIR=/tmp
T=${TAG:-r02final}; mkdir -p gpurun_out/$T
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/$T/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/$T/pytest_gpu.log; echo STOP tests; exit 1; }
tail -1 gpurun_out/$T/pytest_gpu.log
REC=8 bash scripts/gpu_prof.sh $T c3 c4 c2 c2multi || { echo STOP prof; exit 1; }
timeout -k 10 400 python -u bench.py > gpurun_out/$T/bench.json 2> gpurun_out/$T/bench.err || { tail -20 gpurun_out/$T/bench.err; echo STOP bench; exit 1; }
head -c 300 gpurun_out/$T/bench.json
