set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/r04h
timeout -k 10 300 python3 scripts/kbench.py --variants 0:0,93:0,90:0 --workloads c3,c4 --tx --rounds 5 > gpurun_out/r04h/tx_pass1.jsonl 2> gpurun_out/r04h/err || { tail -20 gpurun_out/r04h/err; exit 1; }
cat gpurun_out/r04h/tx_pass1.jsonl
