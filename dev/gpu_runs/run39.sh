#!/bin/bash
# carried retries in the seqlock round kernels: correctness + KV A/B
cd "$(dirname "$0")/../.." || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_arena_gpu.py tests/test_route_gpu.py tests/test_bench_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu39.log 2>&1 || exit 1
for e in "SPLINTER_ARENA_CARRY=1" "SPLINTER_ARENA_CARRY=0" "SPLINTER_ARENA_CARRY=1 SPLINTER_ARENA_UGET=4" "SPLINTER_ARENA_CARRY=1 SPLINTER_ARENA_U=2"; do
  echo "== $e" >> gpurun_out/bench39.log
  env $e timeout -k 10 240 python bench.py --mode kv >> gpurun_out/bench39.log 2>&1 || exit 1
done
echo "== carry keys 16M" >> gpurun_out/bench39.log
timeout -k 10 240 python bench.py --mode kv --keys-per-gpu 16000000 >> gpurun_out/bench39.log 2>&1 || exit 1
echo "== mixed" >> gpurun_out/bench39.log
timeout -k 10 240 python bench.py >> gpurun_out/bench39.log 2>&1
echo "exit=$?"
