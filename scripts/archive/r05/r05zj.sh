#!/bin/bash
# r05zj: the shipped tree at the end of the round: every GPU test, smoke, churn, the bench.
set -u
O=gpurun_out/r05zj; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu tests/ > $O/pytest.log 2>&1 || { echo "STOP pytest"; tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "STOP smoke"; tail -20 $O/smoke.log; exit 1; }
timeout -k 10 120 dpdk-tcpipstack_amd/build/churn_bench 65536 4096 40 10 > $O/churn_65536_10.json 2>&1 || { echo "STOP churn"; cat $O/churn_65536_10.json; exit 1; }
timeout -k 10 400 python3 -u bench.py > $O/bench.json 2> $O/bench.err || { echo "STOP bench"; tail -30 $O/bench.err; exit 1; }
cut -c1-300 $O/churn_65536_10.json
echo r05zj done
