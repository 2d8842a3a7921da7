#!/bin/bash
set -o pipefail
OUT=gpurun_out/r5h
mkdir -p $OUT
timeout -k 10 300 python scripts/encoder_split_ab.py > $OUT/split_ab.jsonl 2> $OUT/split_ab.err || { tail -20 $OUT/split_ab.err; exit 1; }
cat $OUT/split_ab.jsonl
timeout -k 10 300 python scripts/encoder_split_ab.py --vary 1 --parts 1,2 > $OUT/split_ab_vary.jsonl 2> $OUT/split_ab_vary.err || { tail -20 $OUT/split_ab_vary.err; exit 1; }
cat $OUT/split_ab_vary.jsonl
