#!/bin/bash
# fresh-container validation: full GPU suite, smoke, default bench, kernel stats of the bench
cd "$(dirname "$0")/../.." || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu33.log 2>&1 &&
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke33.log 2>&1 &&
timeout -k 10 300 python bench.py > gpurun_out/bench33.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof33 -o run -- python bench.py --steps 5 --warmup 2 > gpurun_out/bench33_prof.log 2>&1
echo "exit=$?"
