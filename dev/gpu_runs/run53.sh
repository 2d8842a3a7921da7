#!/bin/bash
# coalesced lane-op mapping in the carry rounds
cd "$(dirname "$0")/../.." || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_arena_gpu.py tests/test_route_gpu.py tests/test_bench_gpu.py tests/test_search_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu53.log 2>&1 || exit 1
for e in "X=0" "X=1"; do
  echo "== $e kv" >> gpurun_out/bench53.log
  env $e timeout -k 10 240 python bench.py --mode kv >> gpurun_out/bench53.log 2>&1 || exit 1
done
echo "== mixed" >> gpurun_out/bench53.log
timeout -k 10 240 python bench.py >> gpurun_out/bench53.log 2>&1
echo "exit=$?"
