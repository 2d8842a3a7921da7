#!/bin/bash
# attention at 3 waves/SIMD (variant 3) vs 2 (variant 2)
cd "$(dirname "$0")/../.." || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_nomic_gpu.py -x -q -k attention --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu38.log 2>&1 || exit 1
timeout -k 10 300 python scripts/attn_bench.py > gpurun_out/attn38.jsonl 2>&1
echo "exit=$?"
