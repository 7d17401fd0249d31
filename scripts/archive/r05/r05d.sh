#!/bin/bash
# r05d: fused payload forms 5 / 6 / 7 (occupancy 4, hybrid stores) against production and form 2.
set -u
O=gpurun_out/r05d; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python3 -u scripts/fusedbench.py --variants 0,101,105,106,107 --rounds 3 --steps 20 > $O/fused_ab.jsonl 2> $O/fused_ab.err || { echo "STOP fusedbench"; tail -30 $O/fused_ab.err; exit 1; }
echo r05d done
