#!/bin/bash
set -u
O=gpurun_out/r02d; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -5 $O/pytest_gpu.log; echo "pytest rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --no-cpu > $O/bench.log 2>&1; rc=$?; tail -c 3000 $O/bench.log; echo "bench rc=$rc"; exit $rc
