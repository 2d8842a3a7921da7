#!/bin/bash
# search candidate pass: current strided DMA vs a sequential-chunk timing probe (wrong rows, timing only)
set -o pipefail
OUT=gpurun_out/r5seq
mkdir -p $OUT
export TMPDIR=/tmp
for v in base seqprobe; do
  if [ $v = base ]; then unset SPLINTER_HIP_VARIANT; else export SPLINTER_HIP_VARIANT=$v; fi
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/$v -o run -- python3 scripts/search_bench.py --nq 256 --iters 3 > $OUT/$v.out 2> $OUT/$v.err || { tail -20 $OUT/$v.err; exit 1; }
  tail -1 $OUT/$v.out
  python3 scripts/prof_summary.py $OUT/$v/run_results.db --top 8 > $OUT/$v.csv || exit 1
  grep -i "search_mma\|rescore" $OUT/$v.csv | cut -c1-200
done
