#!/bin/bash
# Copy scripts/gpu_final.sh's outputs (gpurun_out/$TAG) into the tracked profiles/$TAG:
# the stamped PMC + trace directories per leg (REC 8 at the top, REC 16 under rec16/), the
# bench command's rocprofv3 stats with its line, the GPU suite and smoke logs, the bench line.
#   bash scripts/collect_profiles.sh RUN_TAG [PROFILE_TAG]     (e.g. r06b r06)
set -eu
TAG=${1:?usage: collect_profiles.sh RUN_TAG [PROFILE_TAG]}
SRC=gpurun_out/$TAG
DST=profiles/${2:-$TAG}
mkdir -p "$DST/rec16" "$DST/bench_cmd" "$DST/check"
for w in c3 c2 c2s c4 c2multi c2multis pf3 pr3 tx3 pg3; do rm -rf "$DST/$w"; cp -r "$SRC/p8/prof/$w" "$DST/"; done
for w in c3 c2 c4 c2multi; do rm -rf "$DST/rec16/$w"; cp -r "$SRC/p16/prof/$w" "$DST/rec16/"; done
cp "$SRC"/final/benchprof/*.csv "$DST/bench_cmd/"
cp "$SRC/final/benchprof.log" "$DST/bench_cmd/bench_under_rocprof.log"
grep '^{' "$SRC/final/benchprof.log" | tail -1 > "$DST/bench_cmd/bench_line.json"
cp "$SRC/final/pytest_gpu.log" "$SRC/final/smoke.log" "$DST/check/"
grep '^{' "$SRC/final/bench.json" | tail -1 > "$DST/bench_line_final_tree.json"
python3 - "$DST" <<'PY'
import json, sys
d = sys.argv[1]
line = json.load(open(f"{d}/bench_cmd/bench_line.json"))
json.dump({k: line[k] for k in ("build", "source_hash", "build_matches_tree")}, open(f"{d}/bench_cmd/build.json", "w"), indent=1)
fin = json.load(open(f"{d}/bench_line_final_tree.json"))
json.dump(fin["cpu_baseline"], open(f"{d}/cpu_baseline.json", "w"), indent=1)
print("bench_cmd", line["build"], "| final line", fin["build"], "traffic_matches_build",
      fin["roofline"]["traffic_matches_build"], "stale", fin["roofline"].get("leg_traffic_files_stale"))
PY
