set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/r04e
timeout -k 10 400 python3 scripts/kbench.py --variants 0:0,91:0,92:0,90:0 --workloads c3,c4,u576 --tx --rounds 5 --check > gpurun_out/r04e/tx_nopipe.jsonl 2> gpurun_out/r04e/tx.err || { tail -20 gpurun_out/r04e/tx.err; exit 1; }
cat gpurun_out/r04e/tx_nopipe.jsonl
