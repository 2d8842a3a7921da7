#!/bin/bash
# KV phase: which batch gets the high-priority queue
cd "$(dirname "$0")/../.." || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
for e in "X=0" "SPLINTER_BENCH_SET_PRIO=high" "X=1" "SPLINTER_BENCH_SET_PRIO=high SPLINTER_ARENA_UGET=4"; do
  echo "== $e kv" >> gpurun_out/bench49.log
  env $e timeout -k 10 240 python bench.py --mode kv >> gpurun_out/bench49.log 2>&1 || exit 1
done
for e in "X=0" "SPLINTER_BENCH_SET_PRIO=high"; do
  echo "== $e mixed" >> gpurun_out/bench49.log
  env $e timeout -k 10 240 python bench.py >> gpurun_out/bench49.log 2>&1 || exit 1
done
echo "exit=$?"
