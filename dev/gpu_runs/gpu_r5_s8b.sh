#!/bin/bash
# 8-wave candidate pass: s_setprio around the MFMA groups / the DMA issued after the first MFMA group,
# against the committed form, interleaved, kernel times
set -o pipefail
OUT=gpurun_out/r5s8b
mkdir -p $OUT
export TMPDIR=/tmp
for r in 1 2; do
  for v in base prio late; do
    if [ $v = base ]; then unset SPLINTER_HIP_VARIANT; else export SPLINTER_HIP_VARIANT=$v; fi
    timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/$v$r -o run -- python3 scripts/search_bench.py --nq 256 --iters 3 > $OUT/$v$r.out 2> $OUT/$v$r.err || { tail -20 $OUT/$v$r.err; exit 1; }
    python3 scripts/prof_summary.py $OUT/$v$r/run_results.db --top 8 > $OUT/$v$r.csv || exit 1
    rm -rf $OUT/$v$r
    echo "$v $r: $(python3 -c "import json; d=json.loads(open('$OUT/$v$r.out').read().strip().splitlines()[-1]); print(round(d['qps']), d['recall_at_k'], d['exact_match'])") pass1 $(grep 'k_search_mma16<1' $OUT/$v$r.csv | awk -F'",' '{print $2}' | cut -d, -f3)"
  done
done
