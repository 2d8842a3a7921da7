# round 2, call 17: post-KV embed slowdown -- clock (GRBM_GUI_ACTIVE cycles vs duration) of k_ln
set -x
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r2_17
mkdir -p $O
cd /tmp
B="--steps 5 --warmup 2 --writer-streams 1 --reader-streams 1 --mop 0 --host-api 0"
timeout -s KILL 200 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_WAVES SQ_BUSY_CYCLES --kernel-include-regex "k_ln" -d $O/cnew -o run -- python3 $GRAFT_REPO_ROOT/bench.py $B > $O/cnew.json 2> $O/cnew.err &&
echo done
