# AVX2 streaming stores for the served staging: server tests, C call-site timing
set -u
export TMPDIR=/tmp
O=gpurun_out/r04al; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_server.py tests/test_c_rx_loop.py tests/test_c_served_latency.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
B=dpdk-tcpipstack_amd/build/served_latency
for args in "64 32 3000" "64 256 2000" "1500 32 3000" "1500 64 2000" "1500 256 1000 1 4" "64 32 3000 1000"; do
  timeout -k 10 120 $B $args >> $O/served_latency.jsonl 2>> $O/err || { tail -5 $O/err; exit 1; }
done
python3 -c "
import json
for l in open('$O/served_latency.jsonl'):
    d=json.loads(l); print(d['frame_bytes'], d['burst'], d['peers'], d['blocks'], 'served', d['served_us']['median'], 'launched', d['launched_us']['median'])
"
