#!/bin/bash
# carried retries + 4-word keys (occupancy) A/B
cd "$(dirname "$0")/../.." || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_arena_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu41.log 2>&1 || exit 1
for e in "X=0" "SPLINTER_ARENA_KW4=1" "X=1" "SPLINTER_ARENA_KW4=1 SPLINTER_ARENA_UGET=4"; do
  echo "== $e" >> gpurun_out/bench41.log
  env $e timeout -k 10 240 python bench.py --mode kv >> gpurun_out/bench41.log 2>&1 || exit 1
done
SPLINTER_ARENA_KW4=1 timeout -k 10 600 python -u -m pytest tests/test_arena_gpu.py -x -q --timeout 300 --timeout-method thread >> gpurun_out/pytest_gpu41.log 2>&1
echo "exit=$?"
