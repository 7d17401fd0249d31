#!/bin/bash
# r05a: bench.py with the RCCL process group at WORLD_SIZE 1 (--pg nccl), the default line
# beside it, then tx / payload-gather re-profiled on this tree (profiles/r05/).
set -u
O=gpurun_out/r05a; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python3 -u bench.py --pg nccl --pg-timeout 300 --steps 20 --warmup 5 > $O/bench_nccl.json 2> $O/bench_nccl.err || { echo "STOP bench nccl"; tail -30 $O/bench_nccl.err; exit 1; }
timeout -k 10 400 python3 -u bench.py --steps 20 --warmup 5 > $O/bench_default.json 2> $O/bench_default.err || { echo "STOP bench default"; tail -30 $O/bench_default.err; exit 1; }
REC=8 bash scripts/gpu_prof.sh r05a tx3 pg3 || exit 1
echo r05a done
