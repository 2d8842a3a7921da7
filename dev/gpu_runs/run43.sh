#!/bin/bash
# set: pulse masks read in the claim re-check (no end-of-round load round trip)
cd "$(dirname "$0")/../.." || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_arena_gpu.py tests/test_route_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu43.log 2>&1 || exit 1
for i in 1 2; do
  echo "== kv $i" >> gpurun_out/bench43.log
  timeout -k 10 240 python bench.py --mode kv >> gpurun_out/bench43.log 2>&1 || exit 1
done
echo "== mixed" >> gpurun_out/bench43.log
timeout -k 10 240 python bench.py >> gpurun_out/bench43.log 2>&1
echo "exit=$?"
