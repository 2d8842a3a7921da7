#!/bin/bash
# stream-posted KV server (SPL_KVS_FUSED=3) vs the fused grid (2): tests, KV-only A/B, mixed step
set -o pipefail
OUT=gpurun_out/r5k
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_arena_gpu.py -k "kvs" > $OUT/tests.txt 2>&1 || { tail -30 $OUT/tests.txt; exit 1; }
tail -3 $OUT/tests.txt
for m in 2 3 2 3; do
  SPL_KVS_FUSED=$m timeout -k 10 400 python bench.py --mode kv --steps 20 --warmup 5 --host-api 0 --host-api-threads2 0 --embed-e2e 0 --daemon-docs 0 --search-keys 0 --exchange-ab 0 --mixed5 0 > $OUT/kv_$m.out 2> $OUT/kv_$m.err || { tail -20 $OUT/kv_$m.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$OUT/kv_$m.out').read().strip().splitlines()[-1]); print($m, d['value'], d['ms_per_step'], d['integrity_failures'], d['timed_set_failures'], d.get('kv_async_error'))"
done
for m in 3 2; do
  SPL_KVS_FUSED=$m timeout -k 10 500 python bench.py --steps 20 --warmup 5 --host-api 0 --host-api-threads2 0 --embed-e2e 0 --daemon-docs 0 --search-keys 0 --exchange-ab 0 --mixed5 0 > $OUT/mixed_$m.out 2> $OUT/mixed_$m.err || { tail -20 $OUT/mixed_$m.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$OUT/mixed_$m.out').read().strip().splitlines()[-1]); print('mixed', $m, d['value'], d['ms_per_step'], d['integrity_failures'], d['timed_set_failures'], d.get('kv_async_error'))"
done
