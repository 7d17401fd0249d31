#!/bin/bash
# GPU-box checks: parity tests, smoke, a short bench and a rocprofv3 kernel-trace summary.
# Every GPU step has its own time limit; a fault/abort/timeout ends the script there.
# Usage: scripts/gpu_check.sh [tag]
set -u
TAG=${1:-r01}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {  # step <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "rc=$rc"; tail -n 25 "$OUT/$name.log"
  case $rc in
    0|1|5) return 0 ;;            # pass / test failures / no tests: GPU still healthy
    *) echo "STOP: $name exited $rc"; exit $rc ;;
  esac
}
rocm-smi --showproductname > "$OUT/rocm-smi.log" 2>&1 || true
step pytest_gpu 600 python -m pytest tests -m gpu -x -q
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench 400 python bench.py --steps 20 --warmup 5
step rocprof 500 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-cpu
echo "=== done"
