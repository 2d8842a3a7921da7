#!/bin/bash
# value rows not a multiple of 16 B: no spill into the neighbour; byte-safe integer ops
cd "$(dirname "$0")/../.." || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_arena_gpu.py tests/test_route_gpu.py -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu54.log 2>&1 || exit 1
timeout -k 10 240 python bench.py --mode kv > gpurun_out/bench54.log 2>&1
echo "exit=$?"
