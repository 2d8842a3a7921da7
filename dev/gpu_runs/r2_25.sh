# round 2, call 25: 32 writer + 32 reader streams vs the hardware-queue budget
set -x
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r2_25
mkdir -p $O
run() { tag=$1; shift; env "$@" timeout -k 10 200 python bench.py --host-api 0 > $O/$tag.json 2> $O/$tag.err; }
run ws32_q1 GPU_MAX_HW_QUEUES=1 &&
run ws32_q2 GPU_MAX_HW_QUEUES=2 &&
run ws32_q3 GPU_MAX_HW_QUEUES=3 &&
run ws32_q4 GPU_MAX_HW_QUEUES=4 &&
echo done
