# A/B: global-address-space pointers (this build) against round 3's library (flat loads and
# stores in the multi-burst kernels and the server)
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/r04l
timeout -k 10 400 python3 scripts/kbench.py --variants 0:0,0:0::dpdk-tcpipstack_amd/rxg/librxg_r03.so --workloads c2m,c4,c3 --rec 8 --rounds 5 --check > gpurun_out/r04l/rec8.jsonl 2> gpurun_out/r04l/rec8.err || { tail -20 gpurun_out/r04l/rec8.err; exit 1; }
grep -v check gpurun_out/r04l/rec8.jsonl; grep -c '"records_equal": true, "counters_equal": true' gpurun_out/r04l/rec8.jsonl
timeout -k 10 300 python3 scripts/kbench.py --variants 0:0,0:0::dpdk-tcpipstack_amd/rxg/librxg_r03.so --workloads c2m --rec 16 --rounds 5 --check > gpurun_out/r04l/rec16.jsonl 2> gpurun_out/r04l/rec16.err || { tail -20 gpurun_out/r04l/rec16.err; exit 1; }
grep -v check gpurun_out/r04l/rec16.jsonl
timeout -k 10 300 python3 scripts/srvlat.py > gpurun_out/r04l/srvlat_new.jsonl 2> gpurun_out/r04l/srvlat_new.err || { tail -20 gpurun_out/r04l/srvlat_new.err; exit 1; }
RXG_LIB=dpdk-tcpipstack_amd/rxg/librxg_r03.so timeout -k 10 300 python3 scripts/srvlat.py > gpurun_out/r04l/srvlat_r03.jsonl 2> gpurun_out/r04l/srvlat_r03.err || { tail -20 gpurun_out/r04l/srvlat_r03.err; exit 1; }
timeout -k 10 300 python3 scripts/srvlat.py > gpurun_out/r04l/srvlat_new2.jsonl 2> gpurun_out/r04l/srvlat_new2.err || exit 1
head -4 gpurun_out/r04l/srvlat_new.jsonl; head -4 gpurun_out/r04l/srvlat_r03.jsonl
