# the reference's call site timed in C (examples/served_latency.c): served and launched bursts + replay
set -u
O=gpurun_out/r04ad; mkdir -p $O
B=dpdk-tcpipstack_amd/build/served_latency
for args in "64 32 2000" "64 1 2000" "64 64 2000" "64 256 1000" "1500 32 2000" "1500 64 2000" "1500 1 2000" "64 32 2000 1000" "1500 32 2000 1000"; do
  timeout -k 10 120 $B $args >> $O/served_latency.jsonl 2>> $O/served_latency.err || { tail -5 $O/served_latency.err; exit 1; }
done
cat $O/served_latency.jsonl
