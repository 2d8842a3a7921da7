#!/bin/bash
# session re-entry check: full GPU suite, smoke(), default bench, kv-only bench
cd "$(dirname "$0")/../.." || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu26.log 2>&1 &&
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke26.log 2>&1 &&
timeout -k 10 400 python bench.py > gpurun_out/bench26.log 2>&1 &&
timeout -k 10 400 python bench.py --mode kv > gpurun_out/bench26_kv.log 2>&1
echo "exit=$?"
