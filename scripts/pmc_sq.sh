#!/bin/bash
# SQ issue/wait breakdown of rx_kernel per workload (one rocprofv3 --pmc pass each).
# Usage: scripts/pmc_sq.sh OUTDIR workload...
set -u
OUT=$1; shift
mkdir -p "$OUT"
export TMPDIR=/tmp
CNT="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_ACTIVE_INST_LDS"
for w in "$@"; do
  timeout -k 10 120 rocprofv3 --pmc $CNT --kernel-include-regex rx_kernel -d "$OUT/$w" -o run --output-format csv \
    -- python3 scripts/kbench.py --variants 0:0 --workloads "$w" --rounds 1 --iters 4 > "$OUT/$w.log" 2>&1
  rc=$?; echo "$w rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
