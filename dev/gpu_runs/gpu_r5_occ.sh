#!/bin/bash
# fused KV grid: workgroups per CU (occupancy) sweep, KV-only bench (100 M keys), two rounds
set -o pipefail
OUT=gpurun_out/r5occ
mkdir -p $OUT
for r in 1 2; do
  for w in 1 2 3; do
    SPL_KVS_FUSED_WG_PER_CU=$w timeout -k 10 300 python bench.py --mode kv --steps 10 --warmup 3 --host-api 0 \
      --host-api-threads2 0 --exchange-ab 0 > $OUT/wpc$w.$r.out 2> $OUT/wpc$w.$r.err || { tail -20 $OUT/wpc$w.$r.err; exit 1; }
    python -c "import json,sys; d=json.loads(open('$OUT/wpc$w.$r.out').read().strip().splitlines()[-1]); print('wpc $w', round(d['value']/1e9,3), 'G', round(d['ms_per_step'],3), 'ms')"
  done
done
