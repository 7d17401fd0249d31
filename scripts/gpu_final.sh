#!/bin/bash
# Round-2 final kernel: rocprofv3 kernel stats + FETCH/WRITE PMC passes (C3, C4, C2, C2 multi-burst)
# and the bench line.
set -u
export TMPDIR=/tmp
REC=8 bash scripts/gpu_prof.sh r02final c3 c4 c2 c2multi || { echo STOP prof; exit 1; }
timeout -k 10 400 python -u bench.py > gpurun_out/r02final/bench.json 2> gpurun_out/r02final/bench.err || { tail -20 gpurun_out/r02final/bench.err; echo STOP bench; exit 1; }
head -c 400 gpurun_out/r02final/bench.json
