# round 2, call 49: 2-rank rehearsal of the routed multi-GPU bench (gloo, both ranks on the one GPU) + the a2a chunk regression
set -x
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r2_49
mkdir -p $O
timeout -k 10 400 python bench.py --gpus 2 --backend gloo --keys-per-gpu 2000000 --batch 1000000 --embed-batch 8 --steps 3 --warmup 1 --host-api 0 --embed-e2e 2 > $O/gloo2.json 2> $O/gloo2.err &&
timeout -k 10 300 python -u -m pytest tests/test_route_gpu.py -x -v --timeout 250 --timeout-method thread > $O/route.log 2>&1 &&
echo done
