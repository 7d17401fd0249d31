#!/bin/bash
# GPU-box checks: parity tests, smoke, the default bench, a rocprofv3 kernel-trace summary
# of the bench's C3 workload and two PMC passes (FETCH_SIZE, WRITE_SIZE) for HBM traffic.
# Every GPU step has its own time limit; a fault/abort/timeout ends the script there.
# Usage: scripts/gpu_check.sh [tag] [steps...]   (steps default: all)
set -u
TAG=${1:-r01}; shift || true
STEPS=${*:-"pytest smoke bench prof pmc pgprof"}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {  # step <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "rc=$rc"; grep -v "amdgpu.ids" "$OUT/$name.log" | tail -n 12
  case $rc in
    0|1|5) return 0 ;;            # pass / test failures / no tests: GPU still healthy
    *) echo "STOP: $name exited $rc"; exit $rc ;;
  esac
}
has() { [[ " $STEPS " == *" $1 "* ]]; }
BENCH_PROF="python3 bench.py --steps 20 --warmup 5 --no-cpu --no-legs"
rocm-smi --showproductname > "$OUT/rocm-smi.log" 2>&1 || true
has pytest && step pytest_gpu 600 python -m pytest tests -m gpu -x -q
has smoke && step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
has bench && step bench 400 python bench.py
has prof && step rocprof 400 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- $BENCH_PROF
has pmc && step pmc_fetch 400 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex rx_kernel -d "$OUT/pmc_fetch" -o run --output-format csv -- $BENCH_PROF
has pmc && step pmc_write 400 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex rx_kernel -d "$OUT/pmc_write" -o run --output-format csv -- $BENCH_PROF
PG="python3 scripts/pgbench.py --workloads c3 --iters 10"
has pgprof && step pg_rocprof 400 rocprofv3 --kernel-trace --stats -d "$OUT/pg_prof" -o run --output-format csv -- $PG
has pgprof && step pg_pmc_fetch 400 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex pg_gather -d "$OUT/pg_pmc_fetch" -o run --output-format csv -- $PG
has pgprof && step pg_pmc_write 400 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex pg_gather -d "$OUT/pg_pmc_write" -o run --output-format csv -- $PG
echo "=== done"
