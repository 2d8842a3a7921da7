# round 2, call 14: bisect the slower post-KV embed phase (ring allocation + descriptor registration)
set -x
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r2_14
mkdir -p $O
B="--writer-streams 1 --reader-streams 1 --mop 1 --host-api 0"
BENCH_SKIP_MOP=1 SPLINTER_HBM_NO_RING=1 timeout -k 10 200 python bench.py $B > $O/noring.json 2> $O/noring.err &&
BENCH_SKIP_MOP=1 timeout -k 10 200 python bench.py $B > $O/ring.json 2> $O/ring.err &&
(cd ab_old && timeout -k 10 200 python bench.py > $O/old.json 2> $O/old.err) &&
echo done
