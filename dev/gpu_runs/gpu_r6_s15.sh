#!/bin/bash
# mode-3 server: occupancy 3 (default build) vs 2 (variant occ2, 2 workgroups per CU, no spills), KV-only
set -o pipefail
OUT=gpurun_out/r6s15
mkdir -p $OUT
KV="--mode kv --steps 20 --warmup 5 --exchange-ab 0 --kv-async-ab 0 --host-api 0 --host-api-threads2 0"
for rep in 1 2 3; do
  for v in default occ2 fused; do
    env_="SPL_KVS_FUSED=3"
    [ $v = occ2 ] && env_="SPL_KVS_FUSED=3 SPLINTER_HIP_VARIANT=occ2 SPL_KVS_FUSED_WG_PER_CU=2"
    [ $v = fused ] && env_="SPL_KVS_FUSED=2"
    env $env_ timeout -k 10 300 python -u bench.py $KV > $OUT/kv_$v.$rep.out 2> $OUT/kv_$v.$rep.err || { tail -20 $OUT/kv_$v.$rep.err; exit 1; }
    python3 -c "import json; d=json.loads([l for l in open('$OUT/kv_$v.$rep.out') if l.startswith('{')][-1]); print('$v rep=$rep', round(d['value']/1e9,4), 'G', round(d['ms_per_step'],3), 'ms integrity', d['integrity_failures'], 'again', d['kv_eagain_retries'], 'err', d.get('kv_async_error'))" | tee -a $OUT/summary.txt
  done
done
