# round 2, call 26: GPU suite + smoke + headline bench (queue budget 2, shared control stream,
# lazy ring stream) + kernel-trace profile
set -x
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r2_26
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 &&
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 &&
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err &&
timeout -k 10 300 python bench.py --mode kv > $O/bench_kv.json 2> $O/bench_kv.err &&
timeout -k 10 300 python bench.py --writer-streams 1 --reader-streams 1 --host-api 0 > $O/bench_ws1.json 2> $O/bench_ws1.err &&
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --host-api 0 > $O/bench_prof.json 2> $O/bench_prof.err &&
echo done
