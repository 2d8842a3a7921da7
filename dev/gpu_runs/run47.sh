#!/bin/bash
# hardware bf16 conversion (v_cvt_pk_bf16_f32) in every GEMM / attention / LN epilogue
cd "$(dirname "$0")/../.." || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_nomic_gpu.py tests/test_search_gpu.py tests/test_splainference.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu47.log 2>&1 || exit 1
timeout -k 10 300 python scripts/gemm_bench.py --tokens 32768 > gpurun_out/gemm47.jsonl 2>&1 || exit 1
timeout -k 10 300 python scripts/attn_bench.py > gpurun_out/attn47.jsonl 2>&1 || exit 1
timeout -k 10 240 python bench.py > gpurun_out/bench47.log 2>&1 || exit 1
timeout -k 10 240 python bench.py --mode embed --embed-batch 512 --steps 5 --warmup 2 > gpurun_out/bench47_embed.log 2>&1
echo "exit=$?"
