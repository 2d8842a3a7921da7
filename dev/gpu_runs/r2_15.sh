# round 2, call 15: bisect the slower post-KV embed phase (round-1 bench.py on this tree's libs)
set -x
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r2_15
mkdir -p $O
timeout -k 10 200 python scripts/bench_r1.py > $O/r1bench_newlib.json 2> $O/r1bench_newlib.err &&
(cd ab_old && timeout -k 10 200 python bench.py > $O/old.json 2> $O/old.err) &&
timeout -k 10 200 python bench.py --writer-streams 1 --reader-streams 1 --mop 0 --host-api 0 > $O/new.json 2> $O/new.err &&
echo done
