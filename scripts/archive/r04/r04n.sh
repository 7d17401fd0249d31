# A/B: global-address-space pointers only in the server (this build) against the commit before
# (librxg_pre.so), multi-burst kernels and server latency
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/r04n
V=0:0,0:0::dpdk-tcpipstack_amd/rxg/librxg_pre.so
timeout -k 10 500 python3 scripts/kbench.py --variants $V --workloads c2m,c2,c4 --rec 8 --rounds 7 --check > gpurun_out/r04n/rec8.jsonl 2> gpurun_out/r04n/rec8.err || { tail -20 gpurun_out/r04n/rec8.err; exit 1; }
grep -v check gpurun_out/r04n/rec8.jsonl; grep -c '"records_equal": true, "counters_equal": true' gpurun_out/r04n/rec8.jsonl
timeout -k 10 300 python3 scripts/kbench.py --variants $V --workloads c2m --rec 16 --rounds 5 > gpurun_out/r04n/rec16.jsonl 2> gpurun_out/r04n/rec16.err || { tail -20 gpurun_out/r04n/rec16.err; exit 1; }
grep -v check gpurun_out/r04n/rec16.jsonl
timeout -k 10 300 python3 scripts/srvlat.py > gpurun_out/r04n/srvlat_new.jsonl 2> gpurun_out/r04n/srvlat_new.err || { tail -20 gpurun_out/r04n/srvlat_new.err; exit 1; }
RXG_LIB=dpdk-tcpipstack_amd/rxg/librxg_pre.so timeout -k 10 300 python3 scripts/srvlat.py > gpurun_out/r04n/srvlat_pre.jsonl 2> gpurun_out/r04n/srvlat_pre.err || { tail -20 gpurun_out/r04n/srvlat_pre.err; exit 1; }
timeout -k 10 300 python3 scripts/srvlat.py > gpurun_out/r04n/srvlat_new2.jsonl 2> gpurun_out/r04n/srvlat_new2.err || exit 1
RXG_LIB=dpdk-tcpipstack_amd/rxg/librxg_pre.so timeout -k 10 300 python3 scripts/srvlat.py > gpurun_out/r04n/srvlat_pre2.jsonl 2> gpurun_out/r04n/srvlat_pre2.err || exit 1
for f in new pre new2 pre2; do echo $f; head -4 gpurun_out/r04n/srvlat_$f.jsonl; done
