# server phase stamps: production (83), no TCB probe (84), hot buckets (86), no search (87), two rounds
set -u
export TMPDIR=/tmp
O=gpurun_out/r04t; mkdir -p $O
for r in 1 2; do for v in 83 84 86 87; do
RXG_LIB=dpdk-tcpipstack_amd/rxg/librxg_exp.so RXG_VARIANT=$v timeout -k 10 200 python3 scripts/srvstamps.py > $O/stamps_${v}_$r.jsonl 2> $O/stamps_${v}_$r.err || { tail -20 $O/stamps_${v}_$r.err; exit 1; }
cat $O/stamps_${v}_$r.jsonl
done; done
