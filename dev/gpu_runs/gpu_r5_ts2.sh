#!/bin/bash
# GEMM tail split inside the encoder: longer interleaved A/B, then a kernel trace of each setting
set -o pipefail
OUT=gpurun_out/r5ts2
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u scripts/gemm_tail_ab.py --rounds 15 > $OUT/tail_ab.jsonl 2> $OUT/tail_ab.err || { tail -20 $OUT/tail_ab.err; exit 1; }
cat $OUT/tail_ab.jsonl
for v in 0 1; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof$v -o run -- python3 scripts/gemm_tail_ab.py --only $v --rounds 3 > $OUT/prof$v.log 2>&1 || { tail -20 $OUT/prof$v.log; exit 1; }
done
find $OUT -name "*kernel_stats.csv" | head
