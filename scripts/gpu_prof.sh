#!/bin/bash
# rocprofv3 evidence per workload: kernel trace + stats, then one PMC pass each for
# FETCH_SIZE and WRITE_SIZE (separate runs: the TCC block holds 4 counters, FETCH_SIZE uses 3,
# WRITE_SIZE 2), converted by scripts/pmc_traffic.py (gfx950: read = 2 x FETCH_SIZE).
# Usage: [REC=8] scripts/gpu_prof.sh TAG WORKLOAD...   (c3 c2 c4 c2multi, tx3 tx4 = tx checksum
# generate, pg3 pg4 = payload gather over C3 / C4, pf3 pf4 = rx + payload fused, pr3 pr4 = the
# fused form by reference; REC: record kind, 16 default)
set -u
TAG=$1; shift
REC=${REC:-16}
export TMPDIR=/tmp
for W in "$@"; do
  O=gpurun_out/$TAG/$W; mkdir -p $O
  CMD="python3 scripts/profrun.py --workload $W --iters 20 --rec $REC"
  case $W in  # the kernel the PMC passes count
    tx*) K="rx_kernel<0," ;;
    pg*) K="pg_gather" ;;
    pf*) K="rx_kernel<$REC, 0, false, false, 1>" ;;
    pr*) K="rx_kernel<$REC, 0, false, false, 2>" ;;
    *)   K="rx_kernel<$REC," ;;
  esac
  # each run writes the build it loaded (src= hash): the trace directory and traffic.json name it
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- $CMD --prov $O/build_trace.json > $O/trace.log 2>&1 || { echo "STOP trace $W"; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$K" -d $O/fetch -o run --output-format csv -- $CMD --prov $O/build_fetch.json > $O/fetch.log 2>&1 || { echo "STOP fetch $W"; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$K" -d $O/write -o run --output-format csv -- $CMD --prov $O/build_write.json > $O/write.log 2>&1 || { echo "STOP write $W"; exit 1; }
  F=$(ls $O/fetch/*counter_collection.csv | head -1); Wr=$(ls $O/write/*counter_collection.csv | head -1)
  python3 scripts/pmc_traffic.py "$F" "$Wr" "$K" $O/traffic.json "$CMD" --prov $O/build_trace.json $O/build_fetch.json $O/build_write.json > /dev/null || { echo "STOP traffic $W"; exit 1; }
  echo "$W ok"
done
echo done
