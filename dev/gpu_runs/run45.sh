#!/bin/bash
# footprint vs throughput at a low-contention batch size (TLB / locality question)
cd "$(dirname "$0")/../.." || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
for k in 2000000 20000000 100000000; do
  for b in 1000000 4000000; do
    echo "== keys $k batch $b" >> gpurun_out/bench45.log
    timeout -k 10 240 python bench.py --mode kv --keys-per-gpu $k --batch $b --steps 20 >> gpurun_out/bench45.log 2>&1 || exit 1
  done
done
echo "exit=$?"
