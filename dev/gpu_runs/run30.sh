#!/bin/bash
# register-epilogue GEMM: persistent (512) vs per-tile (513) vs LDS-epilogue 256/128, encoder shapes + 8192^3
cd "$(dirname "$0")/../.." || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_nomic_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu30.log 2>&1 &&
timeout -k 10 300 python scripts/gemm_bench.py --tokens 32768 > gpurun_out/gemm30.jsonl 2>&1 &&
timeout -k 10 300 python scripts/gemm_bench.py --square 8192 --rounds 3 > gpurun_out/gemm30_sq8k.jsonl 2>&1
echo "exit=$?"
