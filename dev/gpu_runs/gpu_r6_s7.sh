#!/bin/bash
# node search (merged threshold) + maintenance overlap tests, KV home-row prefetch A/B, GPU suite, bench
set -o pipefail
OUT=gpurun_out/r6s7
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_search_gpu.py -k "node_search_batch or search_batch_matches or c_abi" -v -s --timeout 200 --timeout-method thread > $OUT/node.txt 2>&1
rc=$?; grep -E "PASSED|FAILED|single_ms|^E " $OUT/node.txt | cut -c1-400 | tail -12
[ $rc -le 1 ] || exit 1
timeout -k 10 900 python -u -m pytest tests/test_maint_gpu.py -v -s --timeout 300 --timeout-method thread > $OUT/maint.txt 2>&1
rc=$?; grep -E "PASSED|FAILED|^E " $OUT/maint.txt | cut -c1-300 | tail -30; grep -o "overlapped_steps[^r]*" $OUT/maint.txt; grep -o "dead_status[^l]*" $OUT/maint.txt
[ $rc -le 1 ] || exit 1
for rep in 1 2; do
  for pf in 0 1; do
    SPL_KVS_PREFETCH=$pf timeout -k 10 300 python -u bench.py --mode kv --steps 20 --warmup 5 --exchange-ab 0 --kv-async-ab 0 > $OUT/kv_pf$pf.$rep.out 2> $OUT/kv_pf$pf.$rep.err || { tail -20 $OUT/kv_pf$pf.$rep.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open('$OUT/kv_pf$pf.$rep.out').read().strip().splitlines()[-1]); print('pf=$pf rep=$rep', round(d['value']/1e9,4), 'G ops/s', round(d['ms_per_step'],3), 'ms integrity', d.get('integrity_failures'))"
  done
done
timeout -k 10 1200 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.txt 2>&1; echo "suite rc=$?"
tail -12 $OUT/pytest_gpu.txt
timeout -k 10 900 python -u bench.py > $OUT/bench.out 2> $OUT/bench.err || { tail -30 $OUT/bench.err; exit 1; }
tail -c 3000 $OUT/bench.out
