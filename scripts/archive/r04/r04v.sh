# partial all-small slices through the server's small path: server tests, then stamps (83, 88)
# and server latency against the previous commit's library
set -u
export TMPDIR=/tmp
O=gpurun_out/r04v; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_server.py tests/test_gpu_replay.py tests/test_c_rx_loop.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for v in 83 88; do
RXG_LIB=dpdk-tcpipstack_amd/rxg/librxg_exp.so RXG_VARIANT=$v timeout -k 10 200 python3 scripts/srvstamps.py > $O/stamps_$v.jsonl 2> $O/stamps_$v.err || { tail -20 $O/stamps_$v.err; exit 1; }
cat $O/stamps_$v.jsonl
done
for r in 1 2; do
  timeout -k 10 300 python3 scripts/srvlat.py > $O/srvlat_new$r.jsonl 2> $O/srvlat_new$r.err || { tail -20 $O/srvlat_new$r.err; exit 1; }
  RXG_LIB=dpdk-tcpipstack_amd/rxg/librxg_prev.so timeout -k 10 300 python3 scripts/srvlat.py > $O/srvlat_prev$r.jsonl 2> $O/srvlat_prev$r.err || { tail -20 $O/srvlat_prev$r.err; exit 1; }
done
for f in new1 prev1 new2 prev2; do echo $f; python3 -c "
import json
for l in open('$O/srvlat_$f.jsonl'):
    d=json.loads(l); print(d['frame_bytes'], d['n'], 'served', d['served'], 'nr', d['served_nr'], 'dev', d['dev'])
"; done
