#!/bin/bash
# Burst + replay under SYN/FIN churn (examples/churn_bench.c): no churn, host fix-ups and
# device fix-ups.  One JSON line per run into $1 (default stdout).  (Round 1's coarse-marking,
# full-rebuild behaviour, measured through the retired experiment library: HISTORY.md.)
set -u
OUT=${1:-/dev/stdout}
B=dpdk-tcpipstack_amd/build/churn_bench
run() { timeout -k 10 120 "$@" >> "$OUT" || { echo "STOP: $* exited $?"; exit 1; }; }
for nf in 65536 1048576; do
  for burst in 32 4096 65536; do
    steps=$(( burst >= 65536 ? 10 : (burst >= 4096 ? 40 : 400) ))
    run $B $nf $burst $steps 0
    run $B $nf $burst $steps 10
    run $B $nf $burst $steps 10 device
  done
done
echo done
