#!/bin/bash
# round-2 checks: GPU tests, churn and mirror benches
set -u
O=gpurun_out/r02b; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -5 $O/pytest_gpu.log; echo "pytest rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 bash scripts/churnbench.sh $O/churn.jsonl > $O/churn.log 2>&1; rc=$?; tail -3 $O/churn.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/mirrorbench.py > $O/mirror_patch.jsonl 2>$O/mirror_patch.err; rc=$?; [ $rc -eq 0 ] || exit $rc
RXG_LIB=dpdk-tcpipstack_amd/rxg/librxg_exp.so RXG_MIRROR_REBUILD=1 timeout -k 10 400 python scripts/mirrorbench.py > $O/mirror_rebuild.jsonl 2>$O/mirror_rebuild.err; rc=$?
echo "mirror rc=$rc"; exit $rc
