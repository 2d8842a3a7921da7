#!/bin/bash
# stream-posted KV server: where the gap to the fused grid is (kernel time vs post latency)
set -o pipefail
OUT=gpurun_out/r5o
mkdir -p $OUT
ROOT=$(pwd)
export TMPDIR=/tmp
X="--host-api 0 --host-api-threads2 0 --embed-e2e 0 --daemon-docs 0 --search-keys 0 --exchange-ab 0 --mixed5 0"
for cfg in 3:2 2:1 3:1; do
  IFS=: read m sp <<< "$cfg"
  SPL_KVS_FUSED=$m SPL_KVS_ASYNC_SPREAD=$sp timeout -k 10 400 python bench.py --mode kv --steps 20 --warmup 5 $X > $OUT/kv_${m}_$sp.out 2> $OUT/kv_${m}_$sp.err || { tail -20 $OUT/kv_${m}_$sp.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$OUT/kv_${m}_$sp.out').read().strip().splitlines()[-1]); print('$cfg', d['value'], d['ms_per_step'], d['integrity_failures'], d.get('kv_async_error'))"
done
for m in 2 3; do
  SPL_KVS_FUSED=$m timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/$OUT/tr$m -o run -- python3 bench.py --mode kv --steps 5 --warmup 2 $X > $OUT/tr$m.out 2> $OUT/tr$m.err || { tail -20 $OUT/tr$m.err; exit 1; }
  f=$(find $OUT/tr$m -name '*kernel_stats.csv' | head -1)
  head -6 "$f" | cut -c1-160
done
