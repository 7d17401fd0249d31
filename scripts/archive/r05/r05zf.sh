#!/bin/bash
# r05zf: the mirror's patch list carried by the burst launch (large BAR: no patch launch):
# every GPU test, the churn bench, smoke, the bench.
set -u
O=gpurun_out/r05zf; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu tests/ > $O/pytest.log 2>&1 || { echo "STOP pytest"; tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for f in 65536 1048576; do for p in 10 0; do
  timeout -k 10 120 dpdk-tcpipstack_amd/build/churn_bench $f 4096 40 $p > $O/churn_${f}_${p}.json 2>&1 || { echo "STOP churn $f $p"; cat $O/churn_${f}_${p}.json; exit 1; }
done; done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- dpdk-tcpipstack_amd/build/churn_bench 65536 4096 40 10 > $O/trace.log 2>&1 || { echo "STOP trace"; tail -20 $O/trace.log; exit 1; }
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "STOP smoke"; tail -20 $O/smoke.log; exit 1; }
timeout -k 10 400 python3 -u bench.py > $O/bench.json 2> $O/bench.err || { echo "STOP bench"; tail -30 $O/bench.err; exit 1; }
cat $O/churn_*.json | cut -c1-330
echo r05zf done
