#!/bin/bash
# KV throughput vs arena footprint (TLB / locality hypothesis)
cd "$(dirname "$0")/../.." || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
for k in 4000000 16000000 40000000 100000000; do
  echo "== keys $k" >> gpurun_out/bench36.log
  timeout -k 10 240 python bench.py --mode kv --keys-per-gpu $k >> gpurun_out/bench36.log 2>&1 || exit 1
done
echo "== kw4 keys 4000000" >> gpurun_out/bench36.log
SPLINTER_ARENA_KW4=1 timeout -k 10 240 python bench.py --mode kv --keys-per-gpu 4000000 >> gpurun_out/bench36.log 2>&1
echo "exit=$?"
