#!/bin/bash
# routed bench integrity at N=1 on RCCL: sets only / gets only / both
cd "$(dirname "$0")/../.." || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
P=29560
for arg in "--set-frac 0.0" "--set-frac 0.999" "--set-frac 0.5 --steps 0" "--set-frac 0.5"; do
  P=$((P+1))
  echo "== $arg" >> gpurun_out/bench58.log
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port $P bench.py --mode kv --force-routed --warmup 1 --keys-per-gpu 20000000 --batch 4000000 $arg >> gpurun_out/bench58.log 2>&1 || exit 1
done
echo "exit=$?"
