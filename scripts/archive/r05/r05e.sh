#!/bin/bash
# r05e: the fused kernel's payload arena placed at other offsets from the frame pool's channel
# interleave (the arena mirrors the pool's layout, so reads and writes walk in step).
set -u
O=gpurun_out/r05e; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python3 -u scripts/fusedbench.py --variants 106 --workloads c3,c4 --shifts 0,256,4096,65536,1048640,8388608,134217728 --rounds 2 --steps 20 > $O/fused_shift.jsonl 2> $O/fused_shift.err || { echo "STOP fusedbench"; tail -30 $O/fused_shift.err; exit 1; }
echo r05e done
