# round 2, call 18: bisect the post-KV embed slowdown -- round-1 HBM store code in this tree's lib
set -x
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r2_18
mkdir -p $O
B="--writer-streams 1 --reader-streams 1 --mop 0 --host-api 0"
SPLINTER_HIP_VARIANT=oldstore timeout -k 10 200 python bench.py $B > $O/oldstore.json 2> $O/oldstore.err &&
timeout -k 10 200 python bench.py $B > $O/new.json 2> $O/new.err &&
echo done
