# round 2, call 23: fan-out merged into arena_kernels.hip -- mixed step, 1+1 and 32+32 streams
set -x
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r2_23
mkdir -p $O
timeout -k 10 200 python bench.py --writer-streams 1 --reader-streams 1 --host-api 0 > $O/ws1.json 2> $O/ws1.err &&
timeout -k 10 200 python bench.py > $O/ws32.json 2> $O/ws32.err &&
(cd ab_old && timeout -k 10 200 python bench.py > $O/old.json 2> $O/old.err) &&
echo done
