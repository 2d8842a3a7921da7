# round 2, call 95: kernel trace of the e2e embedding loop (GPU busy vs gaps per batch)
set -x
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r2_95
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/prof -o run -- python3 bench.py --mode embed --host-api 0 --steps 2 --warmup 1 --keys-per-gpu 1000000 --embed-e2e 10 > $O/e2e.json 2> $O/e2e.err &&
echo done
