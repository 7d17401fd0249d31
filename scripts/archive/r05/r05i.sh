#!/bin/bash
# r05i: the fused kernel's grid (workgroups; 768 = the occupancy grid, 3 per CU).
set -u
O=gpurun_out/r05i; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python3 -u scripts/fusedbench.py --variants 0,0@256,0@384,0@512,0@640,0@704 --workloads c3,c4 --rounds 3 --steps 20 > $O/fused_grid.jsonl 2> $O/fused_grid.err || { echo "STOP fusedbench"; tail -30 $O/fused_grid.err; exit 1; }
echo r05i done
