#!/bin/bash
# fused KV round: skip the val_len write of same-length updates (SPL_KVS_SKIP_LEN=1) -- tests + KV-only A/B
set -o pipefail
OUT=gpurun_out/r5x
mkdir -p $OUT
SPL_KVS_SKIP_LEN=1 timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_arena_gpu.py > $OUT/tests.txt 2>&1 || { tail -30 $OUT/tests.txt; exit 1; }
tail -2 $OUT/tests.txt
X="--host-api 0 --host-api-threads2 0 --embed-e2e 0 --daemon-docs 0 --search-keys 0 --exchange-ab 0 --mixed5 0"
for sk in 0 1 0 1 0 1; do
  SPL_KVS_SKIP_LEN=$sk timeout -k 10 400 python bench.py --mode kv --steps 20 --warmup 5 $X > $OUT/kv_$sk.out 2> $OUT/kv_$sk.err || { tail -20 $OUT/kv_$sk.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$OUT/kv_$sk.out').read().strip().splitlines()[-1]); print($sk, d['value'], d['ms_per_step'], d['integrity_failures'], d['timed_set_failures'])"
done
