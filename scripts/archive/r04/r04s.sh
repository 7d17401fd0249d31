# inline descriptors for served host bursts of <= 32 frames: server tests, then server latency
# alternating this build and the previous commit's (librxg_prev.so)
set -u
export TMPDIR=/tmp
O=gpurun_out/r04s; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_server.py tests/test_c_rx_loop.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for r in 1 2; do
  timeout -k 10 300 python3 scripts/srvlat.py > $O/srvlat_new$r.jsonl 2> $O/srvlat_new$r.err || { tail -20 $O/srvlat_new$r.err; exit 1; }
  RXG_LIB=dpdk-tcpipstack_amd/rxg/librxg_prev.so timeout -k 10 300 python3 scripts/srvlat.py > $O/srvlat_prev$r.jsonl 2> $O/srvlat_prev$r.err || { tail -20 $O/srvlat_prev$r.err; exit 1; }
done
for f in new1 prev1 new2 prev2; do echo $f; python3 -c "
import json,sys
for l in open('$O/srvlat_$f.jsonl'):
    d=json.loads(l); print(d['frame_bytes'], d['n'], 'served', d['served'], 'nr', d['served_nr'], 'dev', d['dev'], 'hostmbox', d.get('served_hostmbox'))
"; done
