# C call-site timing with the replay split out
set -u
O=gpurun_out/r04ae; mkdir -p $O
B=dpdk-tcpipstack_amd/build/served_latency
for args in "64 32 3000" "64 1 3000" "1500 32 3000" "64 32 3000 1000"; do
  timeout -k 10 120 $B $args >> $O/served_latency.jsonl 2>> $O/served_latency.err || { tail -5 $O/served_latency.err; exit 1; }
done
cat $O/served_latency.jsonl
