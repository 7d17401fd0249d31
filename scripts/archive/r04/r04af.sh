# two cooperative slices: server tests, then C call-site timing of this build and HEAD's
# (LD_LIBRARY_PATH is not used by the example: its rpath names the product library, so the
# previous build runs through a copy of the example linked against librxg_prev.so)
set -u
export TMPDIR=/tmp
O=gpurun_out/r04af; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_server.py tests/test_c_rx_loop.py tests/test_c_served_latency.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
B=dpdk-tcpipstack_amd/build/served_latency
P=dpdk-tcpipstack_amd/build/served_latency_prev
for r in 1 2; do
for args in "64 32 2000" "64 96 2000" "64 128 2000" "1500 32 2000" "1500 96 2000" "1500 128 2000"; do
  timeout -k 10 120 $B $args >> $O/new.jsonl 2>> $O/err || { tail -5 $O/err; exit 1; }
  timeout -k 10 120 $P $args >> $O/prev.jsonl 2>> $O/err || { tail -5 $O/err; exit 1; }
done; done
for f in new prev; do echo $f; python3 -c "
import json
for l in open('$O/$f.jsonl'):
    d=json.loads(l); print(d['frame_bytes'], d['burst'], 'served', d['served_us']['median'])
"; done
