#!/bin/bash
# r05p: the by-reference fused form (messages only, no payload copy) on other grids: it
# runs on the copy form's 2 workgroups per CU today.
set -u
O=gpurun_out/r05p; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python3 -u scripts/fusedbench.py --by-ref --variants 0@512,0@768,0@1024,0@2048 --rounds 3 --steps 20 > $O/byref_grid.jsonl 2> $O/byref_grid.err || { echo "STOP fusedbench"; tail -30 $O/byref_grid.err; exit 1; }
echo r05p done
