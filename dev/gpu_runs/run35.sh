#!/bin/bash
# 4-word keys in the round kernels (occupancy): correctness + KV A/B
cd "$(dirname "$0")/../.." || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_arena_gpu.py tests/test_route_gpu.py tests/test_bench_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu35.log 2>&1 || exit 1
for e in "X=0" "SPLINTER_ARENA_SETOCC=1" "SPLINTER_ARENA_KW16=1" "SPLINTER_ARENA_U=8 SPLINTER_ARENA_UGET=2" "SPLINTER_ARENA_UGET=4"; do
  echo "== $e" >> gpurun_out/bench35.log
  env $e timeout -k 10 240 python bench.py --mode kv >> gpurun_out/bench35.log 2>&1 || exit 1
done
echo "== mixed" >> gpurun_out/bench35.log
timeout -k 10 240 python bench.py >> gpurun_out/bench35.log 2>&1
echo "exit=$?"
