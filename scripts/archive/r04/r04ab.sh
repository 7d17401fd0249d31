# the served body's phases, finer before the first step (variant 88)
set -u
export TMPDIR=/tmp
O=gpurun_out/r04ab; mkdir -p $O
for r in 1 2; do
RXG_LIB=dpdk-tcpipstack_amd/rxg/librxg_exp.so RXG_VARIANT=88 timeout -k 10 200 python3 scripts/srvstamps.py > $O/stamps_88_$r.jsonl 2> $O/stamps_88_$r.err || { tail -20 $O/stamps_88_$r.err; exit 1; }
cat $O/stamps_88_$r.jsonl
done
