# round 2, call 19: bisect the post-KV embed slowdown -- round-1 arena kernels in this tree's lib
set -x
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r2_19
mkdir -p $O
B="--writer-streams 1 --reader-streams 1 --mop 0 --host-api 0"
SPLINTER_HIP_VARIANT=oldkern timeout -k 10 200 python bench.py $B > $O/oldkern.json 2> $O/oldkern.err &&
timeout -k 10 200 python bench.py $B > $O/new.json 2> $O/new.err &&
echo done
