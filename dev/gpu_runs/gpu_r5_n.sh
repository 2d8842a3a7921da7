#!/bin/bash
# stream-posted KV server: spill trim, slice order (spread 1 / 0), chunk size vs the fused grid
set -o pipefail
OUT=gpurun_out/r5p
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_arena_gpu.py -k "kvs" > $OUT/tests.txt 2>&1 || { tail -30 $OUT/tests.txt; exit 1; }
tail -2 $OUT/tests.txt
X="--host-api 0 --host-api-threads2 0 --embed-e2e 0 --daemon-docs 0 --search-keys 0 --exchange-ab 0 --mixed5 0"
for cfg in 2:2048:1 3:2048:1 3:2048:0 2:2048:1 3:2048:1 3:2048:0; do
  IFS=: read m c sp <<< "$cfg"
  SPL_KVS_FUSED=$m SPL_KVS_ASYNC_CHUNK=$c SPL_KVS_ASYNC_SPREAD=$sp timeout -k 10 400 python bench.py --mode kv --steps 20 --warmup 5 $X > $OUT/kv_${m}_${c}_$sp.out 2> $OUT/kv_${m}_${c}_$sp.err || { tail -20 $OUT/kv_${m}_${c}_$sp.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$OUT/kv_${m}_${c}_$sp.out').read().strip().splitlines()[-1]); print('$cfg', d['value'], d['ms_per_step'], d['integrity_failures'], d['timed_set_failures'], d.get('kv_async_error'), d['kv_eagain_retries'])"
done
