#!/bin/bash
# A/B of the software-pipelined streaming-class rounds (experiment variants 42/43) against production.
set -u
O=gpurun_out/pipe; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python3 scripts/kbench.py --variants 0:2048,42:2048,43:2048 --workloads c4,c3,u576,c2,c2m --rec 8 --rounds 5 --check > $O/rec8.jsonl 2> $O/rec8.err || { tail -20 $O/rec8.err; echo STOP rec8; exit 1; }
cat $O/rec8.jsonl
timeout -k 10 300 python3 scripts/kbench.py --variants 0:2048,42:2048 --workloads c4,c3,u576 --tx --rounds 5 > $O/tx.jsonl 2> $O/tx.err || { tail -20 $O/tx.err; echo STOP tx; exit 1; }
cat $O/tx.jsonl
