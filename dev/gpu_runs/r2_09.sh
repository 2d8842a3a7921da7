# round 2, call 9: same box A/B of the mixed step, round-1 tree (ab_old) vs this tree
set -x
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r2_09
mkdir -p $O
(cd ab_old && timeout -k 10 200 python bench.py > $O/old1.json 2> $O/old1.err) &&
timeout -k 10 200 python bench.py --writer-streams 1 --reader-streams 1 --mop 0 --host-api 0 > $O/new1.json 2> $O/new1.err &&
(cd ab_old && timeout -k 10 200 python bench.py > $O/old2.json 2> $O/old2.err) &&
timeout -k 10 200 python bench.py --writer-streams 1 --reader-streams 1 --mop 0 --host-api 0 > $O/new2.json 2> $O/new2.err &&
echo done
