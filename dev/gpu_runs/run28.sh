#!/bin/bash
# persistent register-epilogue GEMM (variant 512): numerics on all variants, A/B vs 256/128/hipBLASLt
cd "$(dirname "$0")/../.." || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_nomic_gpu.py -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu28.log 2>&1 &&
timeout -k 10 300 python scripts/gemm_bench.py --tokens 32768 > gpurun_out/gemm28.jsonl 2>&1
echo "exit=$?"
