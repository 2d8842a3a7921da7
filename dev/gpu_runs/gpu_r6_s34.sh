#!/bin/bash
# LDS-DMA row copies (default) vs register copies: mixed step with the driver's arenas, and config #2's
# server against the fused grid
set -o pipefail
OUT=gpurun_out/r6s34
mkdir -p $OUT
B="--steps 30 --warmup 3 --embed-e2e 0 --host-api 0 --host-api-threads2 0 --daemon-docs 0 --exchange-ab 0 --kv-async-ab 0 --mixed5 0 --search-queries 0"
KV="--mode kv --steps 20 --warmup 5 --exchange-ab 0 --kv-async-ab 0 --host-api 0 --host-api-threads2 0"
for rep in 1 2 3; do
  for c in 0 1; do
    SPL_KVS_COPY_DMA=$c timeout -k 10 500 python -u bench.py $B > $OUT/mix_$c.$rep.out 2> $OUT/mix_$c.$rep.err || { tail -20 $OUT/mix_$c.$rep.err; exit 1; }
    python3 -c "import json; d=json.loads([l for l in open('$OUT/mix_$c.$rep.out') if l.startswith('{')][-1]); print('mixed dma$c rep=$rep', round(d['value']/1e9,4), 'G', round(d['ms_per_step'],3), 'ms integrity', d['integrity_failures'], d['timed_set_failures'], 'again', d['kv_eagain_retries'])" | tee -a $OUT/summary.txt
  done
done
for rep in 1 2; do
  for c in 0 1; do
    SPL_KVS_FUSED=3 SPL_KVS_COPY_DMA=$c timeout -k 10 300 python -u bench.py $KV > $OUT/srv_$c.$rep.out 2> $OUT/srv_$c.$rep.err || { tail -20 $OUT/srv_$c.$rep.err; exit 1; }
    python3 -c "import json; d=json.loads([l for l in open('$OUT/srv_$c.$rep.out') if l.startswith('{')][-1]); print('server dma$c rep=$rep', round(d['value']/1e9,4), 'G', round(d['ms_per_step'],3), 'ms integrity', d['integrity_failures'], d['timed_set_failures'], 'again', d['kv_eagain_retries'])" | tee -a $OUT/summary.txt
  done
done
