#!/bin/bash
# stream-posted KV server: step timeline (kernel trace) + mixed step A/B against the fused grid
set -o pipefail
OUT=gpurun_out/r5q
mkdir -p $OUT
ROOT=$(pwd)
export TMPDIR=/tmp
X="--host-api 0 --host-api-threads2 0 --embed-e2e 0 --daemon-docs 0 --search-keys 0 --exchange-ab 0 --mixed5 0"
SPL_KVS_FUSED=3 timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/$OUT/tr3 -o run -- python3 bench.py --mode kv --steps 8 --warmup 2 $X > $OUT/tr3.out 2> $OUT/tr3.err || { tail -20 $OUT/tr3.err; exit 1; }
for m in 3 2 3 2; do
  SPL_KVS_FUSED=$m timeout -k 10 500 python bench.py --steps 20 --warmup 5 $X > $OUT/mixed_$m.out 2> $OUT/mixed_$m.err || { tail -20 $OUT/mixed_$m.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$OUT/mixed_$m.out').read().strip().splitlines()[-1]); print('mixed', $m, d['value'], d['ms_per_step'], d['integrity_failures'], d['timed_set_failures'], d.get('kv_async_error'), d['config']['writer_streams'])"
done
