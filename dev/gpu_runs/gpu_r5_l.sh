#!/bin/bash
# stream-posted KV server, parallel slice scan: tests, KV-only A/B vs the fused grid, chunk size
set -o pipefail
OUT=gpurun_out/r5m
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_arena_gpu.py -k "kvs" > $OUT/tests.txt 2>&1 || { tail -30 $OUT/tests.txt; exit 1; }
tail -3 $OUT/tests.txt
X="--host-api 0 --host-api-threads2 0 --embed-e2e 0 --daemon-docs 0 --search-keys 0 --exchange-ab 0 --mixed5 0"
for cfg in 2:2048 3:2048 3:4096 2:2048 3:2048 3:4096; do
  m=${cfg%%:*}; c=${cfg##*:}
  SPL_KVS_FUSED=$m SPL_KVS_ASYNC_CHUNK=$c timeout -k 10 400 python bench.py --mode kv --steps 20 --warmup 5 $X > $OUT/kv_${m}_$c.out 2> $OUT/kv_${m}_$c.err || { tail -20 $OUT/kv_${m}_$c.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$OUT/kv_${m}_$c.out').read().strip().splitlines()[-1]); print('$cfg', d['value'], d['ms_per_step'], d['integrity_failures'], d['timed_set_failures'], d.get('kv_async_error'))"
done
