# one shared slice per workgroup (large frames, 3..gridDim slices): server tests, served soak,
# C call-site timing with 4 workgroups against HEAD's build
set -u
export TMPDIR=/tmp
O=gpurun_out/r04ak; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_server.py tests/test_c_served_latency.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
RXG_SOAK=60 timeout -k 10 200 python -u -m pytest tests/test_gpu_soak.py -m gpu -x -q -s -k served --timeout 150 --timeout-method thread > $O/soak.log 2>&1 || { tail -20 $O/soak.log; exit 1; }
tail -3 $O/soak.log
B=dpdk-tcpipstack_amd/build/served_latency
P=dpdk-tcpipstack_amd/build/served_latency_prev
for r in 1 2; do
for args in "1500 160 1500 1 4" "1500 256 1500 1 4" "1500 64 1500 1 4" "64 256 1500 1 4" "1500 256 1500 1 1"; do
  timeout -k 10 120 $B $args >> $O/new.jsonl 2>> $O/err || { tail -5 $O/err; exit 1; }
  timeout -k 10 120 $P $args >> $O/prev.jsonl 2>> $O/err || { tail -5 $O/err; exit 1; }
done; done
for f in new prev; do echo $f; python3 -c "
import json
for l in open('$O/$f.jsonl'):
    d=json.loads(l); print(d['frame_bytes'], d['burst'], 'blocks', d['blocks'], 'served', d['served_us']['median'])
"; done
