#!/bin/bash
# bf16 candidate pass with 64-dim DMA chunks (SPL_SEARCH16_KS=2, 96 KB in flight per CU) vs 32-dim (1)
set -o pipefail
OUT=gpurun_out/r5w
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_search_gpu.py > $OUT/tests.txt 2>&1 || { tail -30 $OUT/tests.txt; exit 1; }
tail -3 $OUT/tests.txt
for cfg in 2:256 1:256 2:512 1:512 2:256 1:256; do
  IFS=: read ks nq <<< "$cfg"
  SPL_SEARCH16_KS=$ks timeout -k 10 300 python scripts/search_bench.py --nq $nq > $OUT/sb_${ks}_$nq.out 2> $OUT/sb_${ks}_$nq.err || { tail -20 $OUT/sb_${ks}_$nq.err; exit 1; }
  python3 -c "import json; d=json.loads([l for l in open('$OUT/sb_${ks}_$nq.out') if l.startswith('{')][-1]); print('$cfg', round(d['qps']), round(d['ms_per_batch'],2), d['recall_at_k'], d['exact_match'], d.get('overflow_queries'))"
done
