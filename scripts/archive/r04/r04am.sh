# AVX2 staging against HEAD's memcpy staging, alternating, C call site
set -u
O=gpurun_out/r04am; mkdir -p $O
B=dpdk-tcpipstack_amd/build/served_latency
P=dpdk-tcpipstack_amd/build/served_latency_prev
for r in 1 2 3; do
for args in "64 32 3000" "1500 32 3000" "64 256 2000" "1500 256 1000 1 4"; do
  timeout -k 10 120 $B $args >> $O/new.jsonl 2>> $O/err || { tail -5 $O/err; exit 1; }
  timeout -k 10 120 $P $args >> $O/prev.jsonl 2>> $O/err || { tail -5 $O/err; exit 1; }
done; done
for f in new prev; do echo $f; python3 -c "
import json
for l in open('$O/$f.jsonl'):
    d=json.loads(l); print(d['frame_bytes'], d['burst'], d['blocks'], 'served', d['served_us']['median'])
"; done
