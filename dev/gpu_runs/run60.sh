#!/bin/bash
# routed set integrity vs all-to-all message size (2 GiB hypothesis)
cd "$(dirname "$0")/../.." || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
TR="python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1"
timeout -k 10 300 $TR --master-port 29581 scripts/route_check.py --mode seq --keys 8388608 > gpurun_out/rc60_8m.log 2>&1
echo "8M rc=$?" >> gpurun_out/rc60_8m.log
timeout -k 10 300 $TR --master-port 29582 scripts/route_check.py --mode seq --keys 16777216 > gpurun_out/rc60_16m.log 2>&1
echo "16M rc=$?" >> gpurun_out/rc60_16m.log
echo done
