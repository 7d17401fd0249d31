#!/bin/bash
# r05za: the replay's counter corrections carried by the next mirror patch launch instead of
# their own counters_add launch: every GPU test, then the churn bench (plain and traced).
set -u
O=gpurun_out/r05za; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu tests/ > $O/pytest.log 2>&1 || { echo "STOP pytest"; tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for f in 65536 1048576; do for p in 10 0; do
  timeout -k 10 120 dpdk-tcpipstack_amd/build/churn_bench $f 4096 40 $p > $O/churn_${f}_${p}.json 2>&1 || { echo "STOP churn $f $p"; cat $O/churn_${f}_${p}.json; exit 1; }
done; done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- dpdk-tcpipstack_amd/build/churn_bench 65536 4096 40 10 > $O/trace.log 2>&1 || { echo "STOP trace"; tail -20 $O/trace.log; exit 1; }
cat $O/churn_*.json
echo r05za done
