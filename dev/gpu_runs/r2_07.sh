# round 2, call 7: kernel traces of the mixed step, 32+32 streams vs 1+1
set -x
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r2_07
mkdir -p $O
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/p32 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --host-api 0 > $O/b32.json 2> $O/b32.err &&
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/p1 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --host-api 0 --writer-streams 1 --reader-streams 1 > $O/b1.json 2> $O/b1.err &&
echo done
