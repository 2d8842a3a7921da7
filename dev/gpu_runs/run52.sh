#!/bin/bash
# cooperative value-row copy in the get rounds too
cd "$(dirname "$0")/../.." || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_arena_gpu.py tests/test_route_gpu.py tests/test_bench_gpu.py tests/test_search_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu52.log 2>&1 || exit 1
for e in "SPLINTER_ARENA_COOP_GET=1" "SPLINTER_ARENA_COOP_GET=0" "SPLINTER_ARENA_COOP_GET=1 X=1" "SPLINTER_ARENA_COOP_GET=0 X=1"; do
  echo "== $e kv" >> gpurun_out/bench52.log
  env $e timeout -k 10 240 python bench.py --mode kv >> gpurun_out/bench52.log 2>&1 || exit 1
done
echo "== mixed" >> gpurun_out/bench52.log
timeout -k 10 240 python bench.py >> gpurun_out/bench52.log 2>&1
echo "exit=$?"
