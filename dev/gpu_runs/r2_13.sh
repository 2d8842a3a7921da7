# round 2, call 13: bisect the slower post-KV embed phase (does using the command ring matter?)
set -x
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r2_13
mkdir -p $O
B="--writer-streams 1 --reader-streams 1 --mop 1 --host-api 0"
BENCH_SKIP_MOP=1 timeout -k 10 200 python bench.py $B > $O/noring.json 2> $O/noring.err &&
timeout -k 10 200 python bench.py $B > $O/ring.json 2> $O/ring.err &&
BENCH_SKIP_MOP=1 timeout -k 10 200 python bench.py $B > $O/noring2.json 2> $O/noring2.err &&
echo done
