# round 2, call 10: kernel traces of the mixed step, round-1 tree vs this tree (same box)
set -x
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r2_10
mkdir -p $O
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/pold -o run -- python3 $GRAFT_REPO_ROOT/ab_old/bench.py --steps 5 --warmup 2 > $O/old.json 2> $O/old.err &&
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/pnew -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --host-api 0 --writer-streams 1 --reader-streams 1 --mop 0 > $O/new.json 2> $O/new.err &&
echo done
