#!/bin/bash
# Pipelined streaming-class rounds as production: GPU tests, A/B against the round-2 form
# (experiment variant 42), bench line.
set -u
O=gpurun_out/${TAG:-pipe2}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; echo STOP tests; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 400 python3 scripts/kbench.py --variants 0:2048,42:2048 --workloads c4,c3,u576,u1500,c2,c2m --rec 8 --rounds 5 --check > $O/rec8.jsonl 2> $O/rec8.err || { tail -20 $O/rec8.err; echo STOP rec8; exit 1; }
cat $O/rec8.jsonl
timeout -k 10 300 python3 scripts/kbench.py --variants 0:2048,42:2048 --workloads c4,c3,u576 --tx --rounds 5 > $O/tx.jsonl 2> $O/tx.err || { tail -20 $O/tx.err; echo STOP tx; exit 1; }
cat $O/tx.jsonl
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; echo STOP bench; exit 1; }
head -c 600 $O/bench.json
