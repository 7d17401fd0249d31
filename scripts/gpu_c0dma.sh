#!/bin/bash
# A/B: class 0 by LDS-DMA computed after the streaming classes (variant 0) vs in the classes' order (44).
set -u
O=gpurun_out/c0dma; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python3 scripts/kbench.py --variants 0:2048,44:2048 --workloads c4,c3,u576,c2 --rec 8 --rounds 5 --check > $O/rec8.jsonl 2> $O/rec8.err || { tail -20 $O/rec8.err; echo STOP rec8; exit 1; }
cat $O/rec8.jsonl
timeout -k 10 300 python3 scripts/kbench.py --variants 0:2048,44:2048 --workloads c4,c3 --tx --rounds 5 > $O/tx.jsonl 2> $O/tx.err || { tail -20 $O/tx.err; echo STOP tx; exit 1; }
cat $O/tx.jsonl
