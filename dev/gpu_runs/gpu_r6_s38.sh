#!/bin/bash
# with the LDS-DMA row copies: fused-grid schedules 2 (wave vote, default), 1 (chunk claims), 0 (barrier)
set -o pipefail
OUT=gpurun_out/r6s38
mkdir -p $OUT
KV="--mode kv --steps 20 --warmup 5 --exchange-ab 0 --kv-async-ab 0 --host-api 0 --host-api-threads2 0"
for rep in 1 2 3; do
  for c in 2 1 0; do
    SPL_KVS_SCHED=$c timeout -k 10 300 python -u bench.py $KV > $OUT/kv_$c.$rep.out 2> $OUT/kv_$c.$rep.err || { tail -20 $OUT/kv_$c.$rep.err; exit 1; }
    python3 -c "import json; d=json.loads([l for l in open('$OUT/kv_$c.$rep.out') if l.startswith('{')][-1]); print('kv sched$c rep=$rep', round(d['value']/1e9,4), 'G', round(d['ms_per_step'],3), 'ms integrity', d['integrity_failures'], d['timed_set_failures'], 'again', d['kv_eagain_retries'])" | tee -a $OUT/summary.txt
  done
done
