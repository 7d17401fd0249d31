#!/bin/bash
# r05z: where the churn bench's burst time goes at 1 % churn (the mirror patch before each
# burst): kernel and HIP API trace of dpdk-tcpipstack_amd/build/churn_bench, 64 K TCBs.
set -u
O=gpurun_out/r05z; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 120 dpdk-tcpipstack_amd/build/churn_bench 65536 4096 40 10 > $O/plain_1pct.json 2>&1 || { echo "STOP plain"; exit 1; }
timeout -k 10 120 dpdk-tcpipstack_amd/build/churn_bench 65536 4096 40 0 > $O/plain_0pct.json 2>&1 || { echo "STOP plain0"; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --hip-trace --stats -d $O/trace -o run --output-format csv -- dpdk-tcpipstack_amd/build/churn_bench 65536 4096 40 10 > $O/trace.log 2>&1 || { echo "STOP trace"; tail -20 $O/trace.log; exit 1; }
cat $O/plain_1pct.json $O/plain_0pct.json
echo r05z done
