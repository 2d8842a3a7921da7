#!/bin/bash
# persistent SwiGLU GEMM (k_gemm256p): numerics, bitwise vs the launch-per-tile kernel, A/B
set -o pipefail
OUT=gpurun_out/r5t
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_nomic_gpu.py -k "gemm256" > $OUT/tests.txt 2>&1 || { tail -30 $OUT/tests.txt; exit 1; }
tail -3 $OUT/tests.txt
timeout -k 10 300 python scripts/gemm256p_ab.py > $OUT/ab.jsonl 2> $OUT/ab.err || { tail -20 $OUT/ab.err; exit 1; }
cat $OUT/ab.jsonl
