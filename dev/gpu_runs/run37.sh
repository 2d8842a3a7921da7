#!/bin/bash
# (1) KV locality headroom: batches pre-sorted by home slot (experiment, untimed sort)
# (2) rcp/exp2 SwiGLU epilogue: GEMM numerics + timings
cd "$(dirname "$0")/../.." || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_nomic_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu37.log 2>&1 || exit 1
timeout -k 10 240 python bench.py --mode kv --presort > gpurun_out/bench37_presort.log 2>&1 || exit 1
timeout -k 10 300 python scripts/gemm_bench.py --tokens 32768 > gpurun_out/gemm37.jsonl 2>&1 || exit 1
timeout -k 10 240 python bench.py > gpurun_out/bench37.log 2>&1
echo "exit=$?"
