#!/bin/bash
# Burst + replay under SYN/FIN churn (examples/churn_bench.c): product library, host and
# device fix-ups, and the round-1 behaviour (experiment library: coarse dport marking, GPU
# fix-ups, full mirror rebuild per sync).  One JSON line per run into $1 (default stdout).
set -u
OUT=${1:-/dev/stdout}
B=dpdk-tcpipstack_amd/build/churn_bench
EXPDIR=$(mktemp -d)
ln -s "$PWD/dpdk-tcpipstack_amd/rxg/librxg_exp.so" "$EXPDIR/librxg.so"
run() { timeout -k 10 120 "$@" >> "$OUT" || { echo "STOP: $* exited $?"; exit 1; }; }
for nf in 65536 1048576; do
  for burst in 32 4096 65536; do
    steps=$(( burst >= 65536 ? 10 : (burst >= 4096 ? 40 : 400) ))
    run $B $nf $burst $steps 0
    run $B $nf $burst $steps 10
    run $B $nf $burst $steps 10 device
    # round 1 (coarse marking, GPU fix-ups, full rebuild per sync) costs O(writes x Ntcb):
    # a few steps, and not the largest burst at 1 M flows
    if [ $nf -lt 1048576 ] || [ $burst -lt 65536 ]; then
      LD_LIBRARY_PATH=$EXPDIR RXG_REPLAY_COARSE=1 RXG_MIRROR_REBUILD=1 run $B $nf $burst 3 10
    fi
  done
done
echo done
