#!/bin/bash
# 16-B coherent probe loads (global_load_dwordx4 sc1) in claim / locate / validate
cd "$(dirname "$0")/../.." || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_arena_gpu.py tests/test_route_gpu.py tests/test_bench_gpu.py tests/test_search_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu46.log 2>&1 || exit 1
for i in 1 2; do
  echo "== kv $i" >> gpurun_out/bench46.log
  timeout -k 10 240 python bench.py --mode kv >> gpurun_out/bench46.log 2>&1 || exit 1
done
echo "== mixed" >> gpurun_out/bench46.log
timeout -k 10 240 python bench.py >> gpurun_out/bench46.log 2>&1 || exit 1
echo "== embed 512" >> gpurun_out/bench46.log
timeout -k 10 240 python bench.py --mode embed --embed-batch 512 --steps 5 --warmup 2 >> gpurun_out/bench46.log 2>&1
echo "exit=$?"
