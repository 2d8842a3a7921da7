#!/bin/bash
# routing overhead on one GPU: the N>1 routed step (RCCL all-to-all with 1 rank) vs the local step
cd "$(dirname "$0")/../.." || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
TR="python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533"
echo "== local kv" >> gpurun_out/bench55.log
timeout -k 10 240 python bench.py --mode kv >> gpurun_out/bench55.log 2>&1 || exit 1
echo "== routed kv" >> gpurun_out/bench55.log
timeout -k 10 300 $TR bench.py --mode kv --force-routed >> gpurun_out/bench55.log 2>&1 || exit 1
echo "== routed mixed" >> gpurun_out/bench55.log
timeout -k 10 300 $TR bench.py --force-routed >> gpurun_out/bench55.log 2>&1 || exit 1
MASTER_ADDR=127.0.0.1 MASTER_PORT=29534 RANK=0 LOCAL_RANK=0 WORLD_SIZE=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof55 -o run -- python bench.py --mode kv --force-routed --steps 5 --warmup 2 > gpurun_out/bench55_prof.log 2>&1
echo "exit=$?"
