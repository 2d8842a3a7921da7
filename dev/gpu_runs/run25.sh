#!/bin/bash
# GEMM tile-order A/B: row-major (GN=0) vs L2 bands (default)
cd "$(dirname "$0")/../.." || exit 1
mkdir -p gpurun_out
NOMIC_GEMM_GN=0 timeout -k 10 300 python scripts/gemm_bench.py --tokens 32768 > gpurun_out/gemm25_rowmajor.jsonl 2>&1 &&
timeout -k 10 300 python scripts/gemm_bench.py --tokens 32768 > gpurun_out/gemm25_band.jsonl 2>&1 &&
NOMIC_GEMM_GN=2 timeout -k 10 300 python scripts/gemm_bench.py --tokens 32768 > gpurun_out/gemm25_band2.jsonl 2>&1
echo "exit=$?"
