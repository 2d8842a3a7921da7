#!/bin/bash
# KV throughput vs value length (is the per-lane row copy the limiter?) + counter list
cd "$(dirname "$0")/../.." || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in 16 64 150 240; do
  echo "== value-len $v" >> gpurun_out/bench50.log
  timeout -k 10 240 python bench.py --mode kv --value-len $v >> gpurun_out/bench50.log 2>&1 || exit 1
done
timeout -s KILL 120 rocprofv3 --list-avail > gpurun_out/avail50.txt 2>&1
echo "exit=$?"
