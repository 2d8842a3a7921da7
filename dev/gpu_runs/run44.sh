#!/bin/bash
# full GPU suite + default bench + kernel stats of the default bench
cd "$(dirname "$0")/../.." || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu44.log 2>&1 || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke44.log 2>&1 || exit 1
timeout -k 10 300 python bench.py > gpurun_out/bench44.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof44 -o run -- python bench.py --steps 5 --warmup 2 > gpurun_out/bench44_prof.log 2>&1
echo "exit=$?"
