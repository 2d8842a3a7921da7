# round 2, call 85: validation of the tree (session 3 end): default bench, kernel profile, full GPU suite, smoke,
# 2-rank routed rehearsal (gloo, one GPU)
set -x
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r2_85
mkdir -p $O
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 bench.py --steps 10 --warmup 2 --host-api 0 --embed-e2e 0 > $O/bench_prof.json 2> $O/bench_prof.err &&
timeout -k 10 800 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 &&
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 &&
timeout -k 10 400 python bench.py --gpus 2 --backend gloo --keys-per-gpu 2000000 --batch 1000000 --embed-batch 8 --steps 3 --warmup 1 --host-api 0 --embed-e2e 2 > $O/gloo2.json 2> $O/gloo2.err &&
echo done
