#!/bin/bash
# kernel stats of the default mixed bench (after the hardware-bf16 epilogues)
cd "$(dirname "$0")/../.." || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof48 -o run -- python bench.py --steps 5 --warmup 2 > gpurun_out/bench48_prof.log 2>&1
echo "exit=$?"
