#!/bin/bash
# r05g: fused kernel time against the payload arena's offset from the frame pool, 16 MiB steps.
set -u
O=gpurun_out/r05g; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python3 -u scripts/fusedbench.py --variants 106 --workloads c3 --shifts 0,16777216,33554432,50331648,67108864,83886080,100663296,117440512,134217728,150994944,167772160,184549376,201326592,218103808,234881024,251658240,268435456,1048640,17825856,34603072,51380288 --rounds 2 --steps 10 > $O/fused_sweep.jsonl 2> $O/fused_sweep.err || { echo "STOP fusedbench"; tail -30 $O/fused_sweep.err; exit 1; }
echo r05g done
