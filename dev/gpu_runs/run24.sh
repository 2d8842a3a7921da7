#!/bin/bash
# full GPU suite + mixed embed/insert/query bench + headline bench
cd "$(dirname "$0")/../.." || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1200 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_gpu24.log 2>&1 &&
timeout -k 10 600 python scripts/mixed_bench.py --slots 8000000 > gpurun_out/mixed24.log 2>&1 &&
timeout -k 10 400 python bench.py > gpurun_out/bench24.log 2>&1
echo "exit=$?"
