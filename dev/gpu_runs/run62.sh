#!/bin/bash
# chunked all-to-all: correctness at 64 MiB - 2.5 GiB, routed set integrity at 8M / 16M keys, routed bench
cd "$(dirname "$0")/../.." || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
TR="python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1"
timeout -k 10 300 $TR --master-port 29601 scripts/a2a_check.py --chunked > gpurun_out/a2a62.log 2>&1
echo "rc=$?" >> gpurun_out/a2a62.log
timeout -k 10 300 $TR --master-port 29602 scripts/route_check.py --mode seq --keys 16777216 > gpurun_out/rc62_16m.log 2>&1
echo "16M rc=$?" >> gpurun_out/rc62_16m.log
timeout -k 10 300 $TR --master-port 29603 scripts/route_check.py --mode pipe --keys 8388608 > gpurun_out/rc62_8m.log 2>&1
echo "8M rc=$?" >> gpurun_out/rc62_8m.log
timeout -k 10 300 $TR --master-port 29604 bench.py --mode kv --force-routed > gpurun_out/bench62_kv.log 2>&1
timeout -k 10 300 $TR --master-port 29605 bench.py --force-routed > gpurun_out/bench62.log 2>&1
echo done
