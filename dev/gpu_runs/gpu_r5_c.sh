#!/bin/bash
# persistent register-epilogue GEMM (gemm_pt.hip): numerics, A/B vs the 256^2 kernel; ring fixes; bench JSON
set -o pipefail
OUT=gpurun_out/r5c
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_nomic_gpu.py -x -v --timeout 120 --timeout-method thread -k "gemm" > $OUT/nomic_gemm.txt 2>&1 || { tail -40 $OUT/nomic_gemm.txt; exit 1; }
tail -2 $OUT/nomic_gemm.txt
timeout -k 10 300 python scripts/gemm_pt_ab.py > $OUT/gemm_pt_ab.jsonl 2> $OUT/gemm_pt_ab.err || { tail -20 $OUT/gemm_pt_ab.err; exit 1; }
cat $OUT/gemm_pt_ab.jsonl
timeout -k 10 300 python -u -m pytest tests/test_ring_gpu.py -x -v --timeout 120 --timeout-method thread -k "owner_close_while or dead_process" > $OUT/ring.txt 2>&1 || { tail -40 $OUT/ring.txt; exit 1; }
tail -2 $OUT/ring.txt
timeout -k 10 700 python bench.py --steps 20 --warmup 5 > $OUT/bench.out 2> $OUT/bench.err || { tail -30 $OUT/bench.err; exit 1; }
tail -1 $OUT/bench.out
grep -E "exchange|integrity" $OUT/bench.err | tail -8
