#!/bin/bash
# In-process A/B of production against experiment variants (kbench, REC8 + tx), records checked.
# Usage: TAG=name VARIANTS=0:2048,63:2048 bash scripts/gpu_ab.sh   (default: this build against
# the round-3 product library kept as rxg/librxg_r03.so)
set -u
O=gpurun_out/${TAG:-ab}; mkdir -p $O
export TMPDIR=/tmp
V=${VARIANTS:-0:0,0:0::dpdk-tcpipstack_amd/rxg/librxg_r03.so}
timeout -k 10 400 python3 scripts/kbench.py --variants $V --workloads ${WLS:-c4,c3,u576,u1500,c2} --rec 8 --rounds 5 --check > $O/rec8.jsonl 2> $O/rec8.err || { tail -20 $O/rec8.err; echo STOP rec8; exit 1; }
grep -v check $O/rec8.jsonl; grep -c '"records_equal": true, "counters_equal": true' $O/rec8.jsonl
timeout -k 10 300 python3 scripts/kbench.py --variants $V --workloads c4,c3,u576 --tx --rounds 5 > $O/tx.jsonl 2> $O/tx.err || { tail -20 $O/tx.err; echo STOP tx; exit 1; }
cat $O/tx.jsonl
