#!/bin/bash
set -u
O=gpurun_out/r02c; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -5 $O/pytest_gpu.log; echo "pytest rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 bash scripts/churnbench.sh $O/churn.jsonl > $O/churn.log 2>&1; rc=$?; tail -3 $O/churn.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/prof_churn -o run --output-format csv -- dpdk-tcpipstack_amd/build/churn_bench 65536 4096 40 10 > $O/prof_churn.log 2>&1; rc=$?
echo "prof rc=$rc"; exit $rc
