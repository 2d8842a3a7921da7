#!/bin/bash
# routed set integrity on RCCL at N=1: sequential vs pipelined phases
cd "$(dirname "$0")/../.." || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
TR="python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1"
timeout -k 10 200 $TR --master-port 29551 scripts/route_check.py --mode seq > gpurun_out/rc57_seq.log 2>&1
echo "seq rc=$?" >> gpurun_out/rc57_seq.log
timeout -k 10 200 $TR --master-port 29552 scripts/route_check.py --mode pipe > gpurun_out/rc57_pipe.log 2>&1
echo "pipe rc=$?" >> gpurun_out/rc57_pipe.log
echo done
