#!/bin/bash
set -u
O=gpurun_out/$1; shift; mkdir -p $O
timeout -k 10 600 python3 scripts/kbench.py "$@" > $O/kbench.jsonl 2> $O/kbench.err; rc=$?
cat $O/kbench.jsonl; tail -3 $O/kbench.err; exit $rc
