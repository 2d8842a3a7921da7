#!/bin/bash
# diagnosis: the fused KV grid with its two cooperative row copies compiled out (variant nocopy:
# results are NOT valid -- values are not moved), an upper bound of what the copy phase costs
set -o pipefail
OUT=gpurun_out/r6s31
mkdir -p $OUT
KV="--mode kv --steps 20 --warmup 5 --exchange-ab 0 --kv-async-ab 0 --host-api 0 --host-api-threads2 0 --verify 0"
for rep in 1 2; do
  for v in default nocopy; do
    E=""; [ $v = nocopy ] && E="SPLINTER_HIP_VARIANT=nocopy"
    env $E timeout -k 10 300 python -u bench.py $KV > $OUT/kv_$v.$rep.out 2> $OUT/kv_$v.$rep.err || { tail -20 $OUT/kv_$v.$rep.err; exit 1; }
    python3 -c "import json; d=json.loads([l for l in open('$OUT/kv_$v.$rep.out') if l.startswith('{')][-1]); print('kv $v rep=$rep', round(d['value']/1e9,4), 'G', round(d['ms_per_step'],3), 'ms again', d['kv_eagain_retries'])" | tee -a $OUT/summary.txt
  done
done
