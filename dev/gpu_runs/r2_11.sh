# round 2, call 11: bisect the slower post-KV embed phase (native fan-out vs python streams)
set -x
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r2_11
mkdir -p $O
B="--writer-streams 1 --reader-streams 1 --mop 0 --host-api 0"
BENCH_PY_STREAMS=1 timeout -k 10 200 python bench.py $B > $O/py.json 2> $O/py.err &&
timeout -k 10 200 python bench.py $B > $O/native.json 2> $O/native.err &&
(cd ab_old && timeout -k 10 200 python bench.py > $O/old.json 2> $O/old.err) &&
echo done
