#!/bin/bash
# Descriptor load at the top of the slice loop (RXG_VARIANT 40/41, experiment library):
# parity on the single-burst GPU tests, then kbench A/B against production.
set -u
O=gpurun_out/dtop; mkdir -p $O
export TMPDIR=/tmp
for V in 40 41; do
RXG_LIB=$PWD/dpdk-tcpipstack_amd/rxg/librxg_exp.so RXG_VARIANT=$V timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_kernel_paths.py tests/test_gpu_fullsize.py -x -q --timeout 120 --timeout-method thread -k "not tx and not replay" > $O/pytest_v$V.log 2>&1
rc=$?; tail -2 $O/pytest_v$V.log; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 600 python3 scripts/kbench.py --variants 0:0,40:0,41:0,32:0 --workloads c4,c3,c2,u576,u1500 --rounds 5 > $O/kb16.jsonl 2> $O/kb16.err || exit 1
cat $O/kb16.jsonl
timeout -k 10 600 python3 scripts/kbench.py --rec 8 --variants 0:0,40:0,41:0 --workloads c4,c3,c2 --rounds 5 > $O/kb8.jsonl 2> $O/kb8.err || exit 1
cat $O/kb8.jsonl
