#!/bin/bash
# GEMM loop throughput at 8192^3 / 4096^3 (long K) for the three kernels vs hipBLASLt
cd "$(dirname "$0")/../.." || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python scripts/gemm_bench.py --square 8192 --rounds 3 > gpurun_out/gemm29_sq8k.jsonl 2>&1 &&
timeout -k 10 300 python scripts/gemm_bench.py --square 4096 --rounds 3 > gpurun_out/gemm29_sq4k.jsonl 2>&1
echo "exit=$?"
