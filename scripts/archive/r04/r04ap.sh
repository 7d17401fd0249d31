# the served body of 32 x 1500 B (class path, four waves) stamped: variant 88, frames of 1500 B
set -u
O=gpurun_out/r04ap; mkdir -p $O
for r in 1 2; do
SRVSTAMPS_FRAME=1500 RXG_LIB=dpdk-tcpipstack_amd/rxg/librxg_exp.so RXG_VARIANT=88 timeout -k 10 200 python3 scripts/srvstamps.py >> $O/stamps_88_1500.jsonl 2>> $O/err || { tail -20 $O/err; exit 1; }
done
python3 -c "
import json
for l in open('$O/stamps_88_1500.jsonl'):
    d=json.loads(l); print(d['case'], {k: d.get(k + '_us') for k in ['args_built','body_entry','all_small_decided','class_rounds_done','class_barrier_passed','class_classified','flushed','counted']}, 'body', d['body_us'], 'host', d['host_us'])
"
