#!/bin/bash
# Deferred phase B experiment (RXG_VARIANT 30-32, experiment library): parity of variant 30
# against the oracle on the single-burst GPU tests, then kbench A/B.
set -u
O=gpurun_out/defer; mkdir -p $O
export TMPDIR=/tmp
RXG_LIB=$PWD/dpdk-tcpipstack_amd/rxg/librxg_exp.so RXG_VARIANT=30 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_kernel_paths.py tests/test_gpu_fullsize.py -x -q --timeout 120 --timeout-method thread -k "not tx and not replay" > $O/pytest_v30.log 2>&1
rc=$?; tail -5 $O/pytest_v30.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python3 scripts/kbench.py --variants 0:0,30:0,32:0,31:0 --workloads c4,c3,c2,u576 --rounds 5 > $O/kb16.jsonl 2> $O/kb16.err || exit 1
cat $O/kb16.jsonl
timeout -k 10 600 python3 scripts/kbench.py --rec 8 --variants 0:0,30:0,32:0 --workloads c4,c3,c2 --rounds 5 > $O/kb8.jsonl 2> $O/kb8.err || exit 1
cat $O/kb8.jsonl
