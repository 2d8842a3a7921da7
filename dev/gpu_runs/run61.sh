#!/bin/bash
# all_to_all_single correctness vs size on RCCL (world 1)
cd "$(dirname "$0")/../.." || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29591 scripts/a2a_check.py > gpurun_out/a2a61.log 2>&1
echo "rc=$?" >> gpurun_out/a2a61.log
echo done
