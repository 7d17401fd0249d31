set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/r04g
timeout -k 10 300 python3 scripts/kbench.py --variants 0:0,13:0,12:0,63:0 --workloads c3,u1500 --rec 8 --rounds 5 > gpurun_out/r04g/c3_phaseb.jsonl 2> gpurun_out/r04g/err || { tail -20 gpurun_out/r04g/err; exit 1; }
cat gpurun_out/r04g/c3_phaseb.jsonl
