#!/bin/bash
# CU-masked overlap of the KV and embed phases: KV on N CUs/XCD, encoder on the rest
cd "$(dirname "$0")/../.." || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
for a in "--kv-cus 8" "--kv-cus 16" "--kv-cus 8 --mode kv" "--kv-cus 16 --mode kv" "--kv-cus 8 --mode embed --embed-batch 64"; do
  echo "== $a" >> gpurun_out/bench34.log
  timeout -k 10 240 python bench.py --steps 10 --warmup 3 $a >> gpurun_out/bench34.log 2>&1 || exit 1
done
echo "exit=$?"
