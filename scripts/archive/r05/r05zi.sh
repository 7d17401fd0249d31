#!/bin/bash
# r05zi: the replay's written-tuple filter on a two-multiply hash: every GPU test, the churn
# bench at both table sizes.
set -u
O=gpurun_out/r05zi; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu tests/ > $O/pytest.log 2>&1 || { echo "STOP pytest"; tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for f in 65536 1048576; do for p in 10 0; do
  timeout -k 10 120 dpdk-tcpipstack_amd/build/churn_bench $f 4096 40 $p > $O/churn_${f}_${p}.json 2>&1 || { echo "STOP churn $f $p"; cat $O/churn_${f}_${p}.json; exit 1; }
done; done
cut -c150-330 $O/churn_*.json
echo r05zi done
