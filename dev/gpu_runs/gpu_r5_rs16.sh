#!/bin/bash
# rescore with 4 candidates in flight per wave vs one (r4w = the 4-wave re-score of the previous commit):
# search GPU tests, then interleaved search_bench rounds with kernel times
set -o pipefail
OUT=gpurun_out/r5rs16
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_search_gpu.py -x -q --timeout 300 --timeout-method thread > $OUT/search_tests.txt 2>&1 || { tail -30 $OUT/search_tests.txt; exit 1; }
tail -1 $OUT/search_tests.txt
for r in 1 2; do
  for v in new r4w; do
    if [ $v = new ]; then unset SPLINTER_HIP_VARIANT; else export SPLINTER_HIP_VARIANT=$v; fi
    timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/$v$r -o run -- python3 scripts/search_bench.py --nq 256 --iters 3 > $OUT/$v$r.out 2> $OUT/$v$r.err || { tail -20 $OUT/$v$r.err; exit 1; }
    python3 scripts/prof_summary.py $OUT/$v$r/run_results.db --top 8 > $OUT/$v$r.csv || exit 1
    rm -rf $OUT/$v$r
    echo "$v $r: $(python3 -c "import json; d=json.loads(open('$OUT/$v$r.out').read().strip().splitlines()[-1]); print(round(d['qps']), d['recall_at_k'], d['exact_match'], round(d['ms_per_batch'],2))") rescore $(grep 'k_rescore' $OUT/$v$r.csv | awk -F'",' '{print $2}' | cut -d, -f3)"
  done
done
