#!/bin/bash
# The one GPU-box driver: each step its own time limit; a fault / abort / timeout (any exit
# other than pass, test failures or no tests) ends the script there, nothing more runs.
#
# Usage: scripts/gpu_check.sh TAG STEP...       (outputs under gpurun_out/TAG/)
#   pytest      the whole -m gpu suite
#   smoke       __graft_entry__.smoke()
#   bench       the default bench line (bench.json)
#   benchprof   rocprofv3 --kernel-trace --stats of the bench command itself (headline only:
#               --no-legs --no-cpu), so its kernel average sits beside the line's kernel_us
#   rehearse    bench.py --gpus 2 (bench.py spawns its 2 ranks itself) on the box's one GPU
#               (gloo collectives; a rehearsal, never a scaling figure)
#   prof        rocprofv3 kernel stats + FETCH_SIZE / WRITE_SIZE passes per workload
#               (scripts/gpu_prof.sh; PROF_WLS, default "c3 c4 c2 c2multi"; REC, default 8)
#   sq          SQ counter passes per workload (scripts/gpu_sq.sh; SQ_WLS)
#   crossover   small-burst crossover against the reference CPU path (scripts/crossover.py)
#   group       group-burst latency (scripts/grouplat.py)
#   churn       burst + replay under SYN/FIN churn (scripts/churnbench.sh)
set -u
TAG=${1:?usage: gpu_check.sh TAG STEP...}; shift
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
    0) return 0 ;;
    1|5) [ "$name" = pytest_gpu ] && { echo "STOP: tests failed"; exit 1; }; return 0 ;;
    *) echo "STOP: $name exited $rc"; exit $rc ;;
  esac
}
rocm-smi --showproductname > "$OUT/rocm-smi.log" 2>&1 || true
for S in "$@"; do
  case $S in
    pytest)    step pytest_gpu 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread ;;
    smoke)     step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()" ;;
    bench)     step bench 500 python -u bench.py; cp "$OUT/bench.log" "$OUT/bench.json" ;;
    benchprof) step benchprof 400 rocprofv3 --kernel-trace --stats -d "$OUT/benchprof" -o run --output-format csv -- python3 -u bench.py --no-legs --no-cpu ;;
    rehearse)  step rehearse2 600 env RXG_BENCH_REHEARSE=1 python3 -u bench.py --gpus 2 --steps 20 --warmup 3 ;;
    prof)      step prof 900 env REC=${REC:-8} bash scripts/gpu_prof.sh "$TAG/prof" ${PROF_WLS:-c3 c4 c2 c2multi} ;;
    sq)        step sq 600 env REC=${REC:-8} bash scripts/gpu_sq.sh ${SQ_WLS:-c4 c3} ;;
    crossover) step crossover 500 python3 -u scripts/crossover.py ;;
    group)     step grouplat 200 python3 -u scripts/grouplat.py ;;
    churn)     step churn 600 bash scripts/churnbench.sh "$OUT/churn.jsonl" ;;
    *) echo "unknown step $S"; exit 2 ;;
  esac
done
echo "=== done"
