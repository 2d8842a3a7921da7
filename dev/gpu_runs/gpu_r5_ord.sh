#!/bin/bash
# KV batch order: random vs sorted by home slot (full sort, then 2^12 / 2^8 buckets)
set -o pipefail
OUT=gpurun_out/r5ord
mkdir -p $OUT
for b in 0 12 8; do
  timeout -k 10 400 python -u scripts/kv_order_ab.py --bucket-bits $b > $OUT/ord_b$b.jsonl 2> $OUT/ord_b$b.err || { tail -20 $OUT/ord_b$b.err; exit 1; }
  cat $OUT/ord_b$b.jsonl
done
