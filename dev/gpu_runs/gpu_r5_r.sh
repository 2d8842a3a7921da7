#!/bin/bash
# routed exchange ordered by device-side posts (flags) vs the gloo collectives: 2-rank tests, exchange A/B
set -o pipefail
OUT=gpurun_out/r5r
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_route_gpu.py tests/test_bench_gpu.py > $OUT/tests.txt 2>&1 || { tail -40 $OUT/tests.txt; exit 1; }
tail -3 $OUT/tests.txt
X="--host-api 0 --host-api-threads2 0 --embed-e2e 0 --daemon-docs 0 --search-keys 0 --mixed5 0"
for sy in flags coll flags; do
  SPLINTER_XR_SYNC=$sy timeout -k 10 900 python bench.py --mode kv --steps 5 --warmup 2 $X --exchange-ab 1 > $OUT/xab_$sy.out 2> $OUT/xab_$sy.err || { tail -20 $OUT/xab_$sy.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$OUT/xab_$sy.out').read().strip().splitlines()[-1]); print('$sy', d['exchange_2rank_ops_per_s'], d['exchange_1rank_ops_per_s'], d['exchange_ratio'], d['exchange_sync'], d['exchange_sync_error'], d['exchange_integrity_failures'], d['exchange_transport'])"
done
