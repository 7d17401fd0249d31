#!/bin/bash
# Round-2 closing evidence for the production kernel: GPU tests, in-process A/B against the
# round-1 descriptor form (variant 32), rocprofv3 stats + PMC passes (REC8), the bench line.
set -u
bash scripts/gpu_tests.sh || exit 1
bash scripts/gpu_kb.sh r02f_ab8 --rec 8 --variants 0:0,32:0 --workloads c2,c2m,c4,c3 --rounds 7 || exit 1
bash scripts/gpu_kb.sh r02f_tx --tx --variants 0:0,32:0 --workloads c3,c4 --rounds 5 || exit 1
REC=8 bash scripts/gpu_prof.sh r02f c3 c2 c4 c2multi || exit 1
timeout -k 10 600 python3 bench.py > gpurun_out/r02f_bench.json 2> gpurun_out/r02f_bench.err || exit 1
tail -c 400 gpurun_out/r02f_bench.json
