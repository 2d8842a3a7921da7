#!/bin/bash
# attention softmax rework (raw exp2, fma scale, masked last tile, deferred rescale) + VGPR-form MFMA
cd "$(dirname "$0")/../.." || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_nomic_gpu.py tests/test_search_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu32.log 2>&1 &&
timeout -k 10 300 python scripts/attn_bench.py > gpurun_out/attn32.jsonl 2>&1 &&
timeout -k 10 300 python scripts/gemm_bench.py --tokens 32768 > gpurun_out/gemm32.jsonl 2>&1 &&
timeout -k 10 300 python bench.py > gpurun_out/bench32.log 2>&1
echo "exit=$?"
