#!/bin/bash
# node-search kernel timeline (rocprofv3 kernel trace), maintenance overlap proof, KV home-row
# prefetch A/B, then the GPU suite and the bench
set -o pipefail
OUT=gpurun_out/r6s5
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/prof_node -o node -- python3 -u -m pytest tests/test_search_gpu.py -k node_search_batch -q -s --timeout 200 > $OUT/prof_node.txt 2>&1
echo "prof rc=$?"; grep -E "single_ms|passed|failed" $OUT/prof_node.txt | cut -c1-300
timeout -k 10 900 python -u -m pytest tests/test_maint_gpu.py -x -v -s --timeout 300 --timeout-method thread > $OUT/maint.txt 2>&1 || { grep -E "PASS|FAIL|^E |overlapped" $OUT/maint.txt | cut -c1-600 | tail -40; exit 1; }
grep -E "PASSED|FAILED" $OUT/maint.txt | cut -c1-200 | tail -30; grep -o "overlapped_steps[^r]*" $OUT/maint.txt; grep -o "dead_status[^l]*" $OUT/maint.txt
for rep in 1 2; do
  for pf in 0 1; do
    SPL_KVS_PREFETCH=$pf timeout -k 10 300 python -u bench.py --mode kv --steps 20 --warmup 5 > $OUT/kv_pf$pf.$rep.out 2> $OUT/kv_pf$pf.$rep.err || { tail -20 $OUT/kv_pf$pf.$rep.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open('$OUT/kv_pf$pf.$rep.out').read().strip().splitlines()[-1]); print('pf=$pf rep=$rep', round(d['value']/1e9,4), 'G ops/s', round(d['ms_per_step'],3), 'ms integrity', d.get('integrity_failures'))"
  done
done
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.txt 2>&1; echo "suite rc=$?"
tail -12 $OUT/pytest_gpu.txt
timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 --embed-e2e 0 --host-api 0 --host-api-threads2 0 --daemon-docs 0 --exchange-ab 0 --mixed5 0 > $OUT/bench.out 2> $OUT/bench.err || { tail -30 $OUT/bench.err; exit 1; }
tail -c 2500 $OUT/bench.out
