#!/bin/bash
# default bench (with the CPU baseline) + a 2-rank rehearsal on the one GPU (gloo collectives)
set -u
O=gpurun_out/r02e; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python bench.py > $O/bench_default.log 2>&1; rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
RXG_BENCH_REHEARSE=1 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 20 --warmup 3 > $O/rehearse2.log 2>&1
rc=$?; echo "rehearse rc=$rc"; tail -c 1500 $O/rehearse2.log; exit $rc
