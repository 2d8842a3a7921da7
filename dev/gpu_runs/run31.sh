#!/bin/bash
# write-through set payload (SPLINTER_ARENA_WT=1, no per-workgroup L2 write-back) vs release fence
cd "$(dirname "$0")/../.." || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_arena_gpu.py tests/test_route_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu31.log 2>&1 &&
SPLINTER_ARENA_WT=0 timeout -k 10 300 python bench.py --mode kv > gpurun_out/bench31_kv_wt0.log 2>&1 &&
SPLINTER_ARENA_WT=1 timeout -k 10 300 python bench.py --mode kv > gpurun_out/bench31_kv_wt1.log 2>&1 &&
SPLINTER_ARENA_WT=0 timeout -k 10 300 python bench.py > gpurun_out/bench31_wt0.log 2>&1 &&
SPLINTER_ARENA_WT=1 timeout -k 10 300 python bench.py > gpurun_out/bench31_wt1.log 2>&1
echo "exit=$?"
