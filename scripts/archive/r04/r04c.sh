set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/r04c
timeout -k 10 300 python -u -m pytest tests/test_gpu_strided.py tests/test_gpu_server.py tests/test_gpu_mirror.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r04c/pytest_new.log 2>&1; rc=$?; tail -15 gpurun_out/r04c/pytest_new.log; [ $rc -eq 0 ] || exit $rc
REC=8 bash scripts/gpu_prof.sh r04c/prof c2s c2multis c2 c2multi c3 c4 || exit 1
timeout -k 10 500 python -u bench.py > gpurun_out/r04c/bench.json 2> gpurun_out/r04c/bench.err || exit 1
python3 -c "
import json; d=json.load(open('gpurun_out/r04c/bench.json'))
print('value', d['value'], d['roofline']['frac'])
for k,v in d['legs'].items():
    if isinstance(v, dict) and 'roofline_frac' in v: print(k, v.get('kernel_us', v.get('kernel_us_per_launch')), v['roofline_frac'])
"
timeout -k 10 400 python3 scripts/kbench.py --variants 0:0,63:0,61:0,60:0,62:0,13:0 --workloads c4,u64 --rec 8 --rounds 5 > gpurun_out/r04c/c4_decomp.jsonl 2> gpurun_out/r04c/c4_decomp.err || { tail -5 gpurun_out/r04c/c4_decomp.err; exit 1; }
cat gpurun_out/r04c/c4_decomp.jsonl
timeout -k 10 120 ./dpdk-tcpipstack_amd/build/txscatter > gpurun_out/r04c/txscatter.jsonl 2>&1 || exit 1
cat gpurun_out/r04c/txscatter.jsonl
