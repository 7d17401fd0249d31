#!/bin/bash
# r05h: on one box -- the copy ceiling (scripts/copybw.hip), the fused forms, and the bench
# (fused leg against the two-pass rx + gather of the same box).
set -u
O=gpurun_out/r05h; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 120 build/copybw 1 2 4 > $O/copybw.jsonl 2> $O/copybw.err || { echo "STOP copybw"; tail -5 $O/copybw.err; exit 1; }
timeout -k 10 400 python3 -u scripts/fusedbench.py --variants 0,106 --workloads c3,c4,c2 --rounds 3 --steps 20 > $O/fused.jsonl 2> $O/fused.err || { echo "STOP fusedbench"; tail -30 $O/fused.err; exit 1; }
timeout -k 10 400 python3 -u bench.py --steps 20 --warmup 5 --no-cpu > $O/bench.json 2> $O/bench.err || { echo "STOP bench"; tail -30 $O/bench.err; exit 1; }
echo r05h done
