set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/r04j
RXG_BENCH_REHEARSE=1 timeout -k 10 600 python3 -u bench.py --gpus 4 --steps 10 --warmup 2 > gpurun_out/r04j/rehearse4.json 2> gpurun_out/r04j/rehearse4.err || { tail -30 gpurun_out/r04j/rehearse4.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/r04j/rehearse4.json'))
print({k: d[k] for k in ('n_gpus','ranks','distinct_devices','collective_backend','counters_ok','value')}, d['cpu_baseline'])
print({k: v.get('counters_ok') for k, v in d['legs'].items() if isinstance(v, dict) and 'counters_ok' in v})
"
