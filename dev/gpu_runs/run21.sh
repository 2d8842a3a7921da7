#!/bin/bash
# batched MFMA search: numerics vs the exact kernel, then QPS/recall at 2M and 25M slots
cd "$(dirname "$0")/../.." || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_search_gpu.py -q -x -k batch > gpurun_out/pytest_search21.log 2>&1 &&
timeout -k 10 300 python scripts/search_bench.py --slots 2000000 --nq 512 > gpurun_out/search21_2m.log 2>&1 &&
timeout -k 10 300 python scripts/search_bench.py --slots 2000000 --nq 1024 >> gpurun_out/search21_2m.log 2>&1 &&
timeout -k 10 600 python scripts/search_bench.py --slots 25000000 --nq 512 > gpurun_out/search21_25m.log 2>&1 &&
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof21 -o search -- python scripts/search_bench.py --slots 25000000 --nq 512 --iters 2 > gpurun_out/search21_prof.log 2>&1
echo "exit=$?"
