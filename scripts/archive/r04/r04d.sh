set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/r04d
timeout -k 10 400 python3 scripts/kbench.py --variants 0:0,90:0,0:0::dpdk-tcpipstack_amd/rxg/librxg_r03.so --workloads c3,c4,u576,c2 --tx --rounds 5 --check > gpurun_out/r04d/tx_two_pass.jsonl 2> gpurun_out/r04d/tx.err || { tail -20 gpurun_out/r04d/tx.err; exit 1; }
cat gpurun_out/r04d/tx_two_pass.jsonl
