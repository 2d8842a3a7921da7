#!/bin/bash
# routed bench integrity at N=1 on RCCL: failing values
cd "$(dirname "$0")/../.." || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29571 bench.py --mode kv --force-routed --warmup 1 --steps 3 --keys-per-gpu 20000000 --batch 4000000 > gpurun_out/bench59.log 2>&1
echo "exit=$?"
