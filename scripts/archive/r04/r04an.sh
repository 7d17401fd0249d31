# the all-small step's tail prefetch in a one-slice served request: stamps 88 against 90, alternating
set -u
O=gpurun_out/r04an; mkdir -p $O
for r in 1 2; do for v in 88 90; do
RXG_LIB=dpdk-tcpipstack_amd/rxg/librxg_exp.so RXG_VARIANT=$v timeout -k 10 200 python3 scripts/srvstamps.py >> $O/stamps_$v.jsonl 2>> $O/err || { tail -20 $O/err; exit 1; }
done; done
for v in 88 90; do python3 -c "
import json
for l in open('$O/stamps_$v.jsonl'):
    d=json.loads(l); print($v, d['case'], 'probe_issued', d['probe_issued_us'], 'classified', d['classified_us'], 'counted', d['counted_us'], 'body', d['body_us'], 'host', d['host_us'])
"; done
