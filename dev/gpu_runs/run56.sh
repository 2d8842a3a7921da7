#!/bin/bash
# routed-step integrity at N=1: which backend / kernel variant
cd "$(dirname "$0")/../.." || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
P=29540
for e in "X=0|--backend nccl" "X=0|--backend gloo" "SPLINTER_ARENA_COOP=0|--backend nccl" "SPLINTER_ARENA_CARRY=0 SPLINTER_ARENA_COOP=0|--backend nccl"; do
  env_=${e%%|*}; arg=${e#*|}; P=$((P+1))
  echo "== $env_ $arg" >> gpurun_out/bench56.log
  env $env_ timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port $P bench.py --mode kv --force-routed --steps 4 --warmup 1 $arg >> gpurun_out/bench56.log 2>&1 || exit 1
done
echo "exit=$?"
