# A/B: global-address-space pointers (this build) against the commit before it (librxg_pre.so,
# built from HEAD~1's rxg_rx.h) and round 3's library, same process, interleaved rounds
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/r04m
V=0:0,0:0::dpdk-tcpipstack_amd/rxg/librxg_pre.so,0:0::dpdk-tcpipstack_amd/rxg/librxg_r03.so
timeout -k 10 500 python3 scripts/kbench.py --variants $V --workloads c2m,c4,c3,c2 --rec 8 --rounds 7 --check > gpurun_out/r04m/rec8.jsonl 2> gpurun_out/r04m/rec8.err || { tail -20 gpurun_out/r04m/rec8.err; exit 1; }
grep -v check gpurun_out/r04m/rec8.jsonl; grep -c '"records_equal": true, "counters_equal": true' gpurun_out/r04m/rec8.jsonl
timeout -k 10 300 python3 scripts/kbench.py --variants $V --workloads c2m --rec 16 --rounds 5 > gpurun_out/r04m/rec16.jsonl 2> gpurun_out/r04m/rec16.err || { tail -20 gpurun_out/r04m/rec16.err; exit 1; }
grep -v check gpurun_out/r04m/rec16.jsonl
timeout -k 10 300 python3 scripts/srvlat.py > gpurun_out/r04m/srvlat_new.jsonl 2> gpurun_out/r04m/srvlat_new.err || { tail -20 gpurun_out/r04m/srvlat_new.err; exit 1; }
RXG_LIB=dpdk-tcpipstack_amd/rxg/librxg_pre.so timeout -k 10 300 python3 scripts/srvlat.py > gpurun_out/r04m/srvlat_pre.jsonl 2> gpurun_out/r04m/srvlat_pre.err || { tail -20 gpurun_out/r04m/srvlat_pre.err; exit 1; }
timeout -k 10 300 python3 scripts/srvlat.py > gpurun_out/r04m/srvlat_new2.jsonl 2> gpurun_out/r04m/srvlat_new2.err || exit 1
RXG_LIB=dpdk-tcpipstack_amd/rxg/librxg_pre.so timeout -k 10 300 python3 scripts/srvlat.py > gpurun_out/r04m/srvlat_pre2.jsonl 2> gpurun_out/r04m/srvlat_pre2.err || exit 1
for f in new pre new2 pre2; do echo $f; head -4 gpurun_out/r04m/srvlat_$f.jsonl; done
