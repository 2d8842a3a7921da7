#!/bin/bash
# get output rows written through the next 64-B boundary (SPL_KVS_PAD_OUT=1: the row's last line whole,
# zeros past the value) vs exactly the value's 16-B chunks (0); tests under 1 first
set -o pipefail
OUT=gpurun_out/r6s39
mkdir -p $OUT
SPL_KVS_PAD_OUT=1 timeout -k 10 600 python -u -m pytest tests/test_arena_gpu.py tests/test_route_gpu.py -x -q --timeout 300 --timeout-method thread > $OUT/tests.txt 2>&1 || { tail -30 $OUT/tests.txt; exit 1; }
tail -1 $OUT/tests.txt
KV="--mode kv --steps 20 --warmup 5 --exchange-ab 0 --kv-async-ab 0 --host-api 0 --host-api-threads2 0"
B="--steps 30 --warmup 3 --embed-e2e 0 --host-api 0 --host-api-threads2 0 --daemon-docs 0 --exchange-ab 0 --kv-async-ab 0 --mixed5 0 --search-queries 0"
for rep in 1 2 3; do
  for c in 0 1; do
    SPL_KVS_PAD_OUT=$c timeout -k 10 300 python -u bench.py $KV > $OUT/kv_$c.$rep.out 2> $OUT/kv_$c.$rep.err || { tail -20 $OUT/kv_$c.$rep.err; exit 1; }
    python3 -c "import json; d=json.loads([l for l in open('$OUT/kv_$c.$rep.out') if l.startswith('{')][-1]); print('kv pad$c rep=$rep', round(d['value']/1e9,4), 'G', round(d['ms_per_step'],3), 'ms integrity', d['integrity_failures'], d['timed_set_failures'], 'again', d['kv_eagain_retries'])" | tee -a $OUT/summary.txt
  done
done
for rep in 1 2; do
  for c in 0 1; do
    SPL_KVS_PAD_OUT=$c timeout -k 10 500 python -u bench.py $B > $OUT/mix_$c.$rep.out 2> $OUT/mix_$c.$rep.err || { tail -20 $OUT/mix_$c.$rep.err; exit 1; }
    python3 -c "import json; d=json.loads([l for l in open('$OUT/mix_$c.$rep.out') if l.startswith('{')][-1]); print('mixed pad$c rep=$rep', round(d['value']/1e9,4), 'G', round(d['ms_per_step'],3), 'ms integrity', d['integrity_failures'], d['timed_set_failures'], 'again', d['kv_eagain_retries'])" | tee -a $OUT/summary.txt
  done
done
