#!/bin/bash
# Payload gather A/B (pgbench, experiment library), payload bytes checked against production.
set -u
O=gpurun_out/${TAG:-pg}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python3 scripts/pgbench.py --variants ${VARIANTS:-0,14} --workloads c3,c4,c2 --iters 20 --check > $O/pg.jsonl 2> $O/pg.err || { tail -20 $O/pg.err; echo STOP pg; exit 1; }
cat $O/pg.jsonl
