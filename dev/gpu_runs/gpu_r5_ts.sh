#!/bin/bash
# GEMM tail split: A/B on the qkv projection and the encoder, then the encoder numerics tests
set -o pipefail
OUT=gpurun_out/r5ts
mkdir -p $OUT
timeout -k 10 300 python -u scripts/gemm_tail_ab.py > $OUT/tail_ab.jsonl 2> $OUT/tail_ab.err || { tail -20 $OUT/tail_ab.err; exit 1; }
cat $OUT/tail_ab.jsonl
timeout -k 10 600 python -u -m pytest tests/test_nomic_gpu.py -x -q --timeout 300 --timeout-method thread > $OUT/nomic_tests.txt 2>&1 || { tail -30 $OUT/nomic_tests.txt; exit 1; }
tail -2 $OUT/nomic_tests.txt
