#!/bin/bash
# side region: probe stats / rehash / bf16 copy tests, batched search on the bf16 copy; GEMM K-sweep
set -o pipefail
OUT=gpurun_out/r5e
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_maint_gpu.py -x -v --timeout 120 --timeout-method thread > $OUT/maint.txt 2>&1 || { tail -40 $OUT/maint.txt; exit 1; }
grep -E "passed|failed|before" $OUT/maint.txt | tail -4
timeout -k 10 400 python -u -m pytest tests/test_search_gpu.py tests/test_arena_gpu.py tests/test_node_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/search_arena.txt 2>&1 || { tail -40 $OUT/search_arena.txt; exit 1; }
tail -2 $OUT/search_arena.txt
timeout -k 10 300 python scripts/search_bench.py > $OUT/search_bench.out 2>&1 || { tail -20 $OUT/search_bench.out; exit 1; }
tail -5 $OUT/search_bench.out
timeout -k 10 300 python scripts/gemm_pt_ab.py --ksweep 1 --encoder 0 > $OUT/gemm_pt_ab.jsonl 2> $OUT/gemm_pt_ab.err || { tail -20 $OUT/gemm_pt_ab.err; exit 1; }
cat $OUT/gemm_pt_ab.jsonl
