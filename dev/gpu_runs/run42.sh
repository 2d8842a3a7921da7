#!/bin/bash
# overlapped KV || embed with fence-free seqlock variants (sc1 payload, no L2 write-back / invalidate)
cd "$(dirname "$0")/../.." || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
for e in "X=0|" "X=0|--overlap" "SPLINTER_ARENA_WT=1 SPLINTER_ARENA_CARRY=0|--overlap" "SPLINTER_ARENA_U=1 SPLINTER_ARENA_MO=1|--overlap" "SPLINTER_ARENA_U=1 SPLINTER_ARENA_MO=1|--mode kv" "SPLINTER_ARENA_U=1 SPLINTER_ARENA_MO=1|"; do
  env_=${e%%|*}; arg=${e#*|}
  echo "== $env_ $arg" >> gpurun_out/bench42.log
  env $env_ timeout -k 10 240 python bench.py $arg >> gpurun_out/bench42.log 2>&1 || exit 1
done
echo "exit=$?"
