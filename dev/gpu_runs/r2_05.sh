# round 2, call 5: 32 writer / 32 reader streams vs the HIP runtime's hardware-queue count
set -x
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r2_05
mkdir -p $O
run() { tag=$1; shift; timeout -k 10 200 python bench.py "$@" > $O/$tag.json 2> $O/$tag.err; }
GPU_MAX_HW_QUEUES=8 run kv_q8 --mode kv &&
GPU_MAX_HW_QUEUES=16 run kv_q16 --mode kv &&
GPU_MAX_HW_QUEUES=32 run kv_q32 --mode kv &&
GPU_MAX_HW_QUEUES=16 run mixed_q16 &&
GPU_MAX_HW_QUEUES=32 run mixed_q32 &&
echo done
