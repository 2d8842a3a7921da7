#!/bin/bash
# mode-3 (stream-posted server) chunk size sweep, KV-only, against the fused grid
set -o pipefail
OUT=gpurun_out/r6s11c
mkdir -p $OUT
KV="--mode kv --steps 20 --warmup 5 --exchange-ab 0 --kv-async-ab 0 --host-api 0 --host-api-threads2 0"
for rep in 1 2; do
  for c in fused 1024 2048 4096; do
    if [ $c = fused ]; then env_="SPL_KVS_FUSED=2"; else env_="SPL_KVS_FUSED=3 SPL_KVS_ASYNC_CHUNK=$c"; fi
    env $env_ timeout -k 10 300 python -u bench.py $KV > $OUT/kv_$c.$rep.out 2> $OUT/kv_$c.$rep.err || { tail -20 $OUT/kv_$c.$rep.err; exit 1; }
    python3 -c "import json; d=json.loads([l for l in open('$OUT/kv_$c.$rep.out') if l.startswith('{')][-1]); print('$c rep=$rep', round(d['value']/1e9,4), 'G', round(d['ms_per_step'],3), 'ms integrity', d['integrity_failures'], 'again', d['kv_eagain_retries'], 'err', d.get('kv_async_error'))"
  done
done
