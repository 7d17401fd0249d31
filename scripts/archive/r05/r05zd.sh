#!/bin/bash
# r05zd: the read ceiling of the headline's access pattern (scripts/readbw_rot.hip, built on the
# box): 16 B/lane streaming reads of two rotating 1.5 GiB buffers.
set -u
O=gpurun_out/r05zd; mkdir -p $O
timeout -k 10 200 /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -o /tmp/readbw_rot scripts/readbw_rot.hip > $O/build.log 2>&1 || { echo "STOP build"; cat $O/build.log; exit 1; }
timeout -k 10 200 /tmp/readbw_rot > $O/readbw.jsonl 2>&1 || { echo "STOP readbw"; cat $O/readbw.jsonl; exit 1; }
cat $O/readbw.jsonl
echo r05zd done
