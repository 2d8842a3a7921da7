#!/bin/bash
# routed C1 fast path: route kernels vs torch reference, segmented set/get, 2-rank gloo rehearsal, arena suite
cd "$(dirname "$0")/../.." || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_route_gpu.py tests/test_arena_gpu.py tests/test_bench_gpu.py -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu27.log 2>&1 &&
timeout -k 10 300 python bench.py --mode kv > gpurun_out/bench27_kv.log 2>&1
echo "exit=$?"
