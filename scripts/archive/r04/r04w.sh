# the served body run twice per request (experiment variant 89): a warm second body
set -u
export TMPDIR=/tmp
O=gpurun_out/r04w; mkdir -p $O
for r in 1 2; do
RXG_LIB=dpdk-tcpipstack_amd/rxg/librxg_exp.so RXG_VARIANT=89 timeout -k 10 200 python3 scripts/srvstamps.py > $O/stamps_89_$r.jsonl 2> $O/stamps_89_$r.err || { tail -20 $O/stamps_89_$r.err; exit 1; }
cat $O/stamps_89_$r.jsonl
done
