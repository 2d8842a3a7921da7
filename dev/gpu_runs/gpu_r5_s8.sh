#!/bin/bash
# 8-wave bf16 candidate pass (query fragments by LDS-DMA): search GPU tests, then A/B against the
# 4-wave pass (libsplinter_hip_s4.so, built from the previous commit), interleaved, kernel times
set -o pipefail
OUT=gpurun_out/r5s8
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_search_gpu.py -x -q --timeout 300 --timeout-method thread > $OUT/search_tests.txt 2>&1 || { tail -30 $OUT/search_tests.txt; exit 1; }
tail -2 $OUT/search_tests.txt
for r in 1 2; do
  for v in new s4; do
    if [ $v = new ]; then unset SPLINTER_HIP_VARIANT; else export SPLINTER_HIP_VARIANT=$v; fi
    timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/$v$r -o run -- python3 scripts/search_bench.py --nq 256 --iters 3 > $OUT/$v$r.out 2> $OUT/$v$r.err || { tail -20 $OUT/$v$r.err; exit 1; }
    python3 scripts/prof_summary.py $OUT/$v$r/run_results.db --top 8 > $OUT/$v$r.csv || exit 1
    rm -rf $OUT/$v$r
    echo "$v $r: $(python3 -c "import json; d=json.loads(open('$OUT/$v$r.out').read().strip().splitlines()[-1]); print(round(d['qps']), d['recall_at_k'], d['exact_match'], d['candidates_per_query'])") pass1 $(grep 'k_search_mma16<1' $OUT/$v$r.csv | awk -F'",' '{print $2}' | cut -d, -f3) pass0 $(grep 'k_search_mma16<0' $OUT/$v$r.csv | awk -F'",' '{print $2}' | cut -d, -f3)"
  done
done
for v in new s4; do
  if [ $v = new ]; then unset SPLINTER_HIP_VARIANT; else export SPLINTER_HIP_VARIANT=$v; fi
  timeout -k 10 400 python3 scripts/search_bench.py --nq 512 --iters 3 > $OUT/${v}_512.out 2> $OUT/${v}_512.err || { tail -20 $OUT/${v}_512.err; exit 1; }
  echo "$v nq512: $(python3 -c "import json; d=json.loads(open('$OUT/${v}_512.out').read().strip().splitlines()[-1]); print(round(d['qps']), d['recall_at_k'], d['exact_match'])")"
done
