#!/bin/bash
# SQ counters (one pass, 8 SQ counters) of the production rx kernel per workload.
set -u
export TMPDIR=/tmp
REC=${REC:-8}
for W in "$@"; do
  O=gpurun_out/sq/$W; mkdir -p $O
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES --kernel-include-regex "rx_kernel<$REC," -d $O -o run --output-format csv -- python3 scripts/profrun.py --workload $W --iters 5 --rec $REC > $O/log 2>&1 || { echo "STOP $W"; tail -5 $O/log; exit 1; }
  # second pass: where the wave cycles go (WAIT_ANY + WAIT_INST_ANY + ACTIVE_INST_ANY = WAVE_CYCLES)
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA --kernel-include-regex "rx_kernel<$REC," -d $O/p2 -o run --output-format csv -- python3 scripts/profrun.py --workload $W --iters 5 --rec $REC > $O/log2 2>&1 || { echo "STOP2 $W"; tail -5 $O/log2; exit 1; }
  echo "$W ok"
done
