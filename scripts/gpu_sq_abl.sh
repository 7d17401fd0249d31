#!/bin/bash
# SQ instruction counts of the REC16 rx kernel and its timing ablations on C4 (experiment
# variants 11 no probe, 12 no record stores, 13 no phase B): where the slice's instructions go.
set -u
O=gpurun_out/sqabl; mkdir -p $O
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES --kernel-include-regex "rx_kernel<16," -d $O/pmc -o run --output-format csv -- python3 scripts/kbench.py --variants 0:0,11:0,12:0,13:0 --workloads c4 --rec 16 --rounds 1 --iters 3 > $O/run.log 2>&1 || { tail -20 $O/run.log; echo STOP; exit 1; }
python3 - <<'PY'
import csv, glob, collections
f = glob.glob('gpurun_out/sqabl/pmc/*counter_collection.csv')[0]
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for r in csv.DictReader(open(f)):
    agg[r['Kernel_Name'][:80]][r['Counter_Name']].append(float(r['Counter_Value']))
for k, d in agg.items():
    print(k, {c: round(sum(v) / len(v)) for c, v in d.items()})
PY
