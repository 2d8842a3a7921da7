#!/bin/bash
# carried-retry kernels: workgroup size / ops-per-lane sweep
cd "$(dirname "$0")/../.." || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
for e in "X=0" "SPLINTER_ARENA_BLOCK=512" "SPLINTER_ARENA_BLOCK=512 SPLINTER_ARENA_BLOCK_GET=256" "SPLINTER_ARENA_BLOCK_GET=512" "SPLINTER_ARENA_UGET=4" "SPLINTER_ARENA_BLOCK=512 SPLINTER_ARENA_U=2 SPLINTER_ARENA_BLOCK_GET=256" "X=1"; do
  echo "== $e" >> gpurun_out/bench40.log
  env $e timeout -k 10 240 python bench.py --mode kv >> gpurun_out/bench40.log 2>&1 || exit 1
done
echo "exit=$?"
