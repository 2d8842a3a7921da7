#!/bin/bash
set -o pipefail
OUT=gpurun_out/r5d
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_nomic_gpu.py -x -q --timeout 120 --timeout-method thread -k "gemm_pt" > $OUT/nomic_pt.txt 2>&1 || { tail -40 $OUT/nomic_pt.txt; exit 1; }
tail -2 $OUT/nomic_pt.txt
timeout -k 10 300 python scripts/gemm_pt_ab.py --ksweep 1 --encoder 1 > $OUT/gemm_pt_ab.jsonl 2> $OUT/gemm_pt_ab.err || { tail -20 $OUT/gemm_pt_ab.err; exit 1; }
cat $OUT/gemm_pt_ab.jsonl
