#!/bin/bash
# exchange pack kernel: value chunks copied 8 per lane in flight (default) vs one load -> store pair at a
# time (variant xserial); route tests first, then the bench's exchange A/B (2 ranks vs 1 on this GPU)
set -o pipefail
OUT=gpurun_out/r6s35
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_route_gpu.py -x -q --timeout 300 --timeout-method thread > $OUT/tests.txt 2>&1 || { tail -30 $OUT/tests.txt; exit 1; }
tail -1 $OUT/tests.txt
X="--mode kv --steps 3 --warmup 1 --host-api 0 --host-api-threads2 0 --kv-async-ab 0 --exchange-ab 1"
for rep in 1 2 3; do
  for v in default xserial; do
    E=""; [ $v = xserial ] && E="SPLINTER_HIP_VARIANT=xserial"
    env $E timeout -k 10 600 python -u bench.py $X > $OUT/x_$v.$rep.out 2> $OUT/x_$v.$rep.err || { tail -20 $OUT/x_$v.$rep.err; exit 1; }
    python3 -c "import json; d=json.loads([l for l in open('$OUT/x_$v.$rep.out') if l.startswith('{')][-1]); print('xch $v rep=$rep', round((d['exchange_2rank_ops_per_s'] or 0)/1e9,4), 'G vs', round((d['exchange_1rank_ops_per_s'] or 0)/1e9,4), 'ratio', round(d['exchange_ratio'] or 0,4), 'integrity', d['exchange_integrity_failures'], d['exchange_transport'])" | tee -a $OUT/summary.txt
  done
done
