#!/bin/bash
# The round's evidence on the shipped tree, in one GPU call: the GPU suite, smoke, rocprofv3 of
# the bench command, the stamped PMC passes of every leg the bench line cites (REC 8 and 16), and
# the default bench line.  Outputs under gpurun_out/$TAG/; scripts/collect_profiles.sh copies
# them into profiles/.  Stops at the first failing step (gpu_check.sh).
#   bash scripts/gpu_final.sh r06
set -eu
TAG=${1:?usage: gpu_final.sh TAG}
bash scripts/gpu_check.sh "$TAG/final" pytest smoke benchprof
PROF_WLS="c3 c2 c2s c4 c2multi c2multis pf3 pr3 tx3 pg3" REC=8 bash scripts/gpu_check.sh "$TAG/p8" prof
PROF_WLS="c3 c2 c4 c2multi" REC=16 bash scripts/gpu_check.sh "$TAG/p16" prof
bash scripts/gpu_check.sh "$TAG/final" bench
