# round 2, call 91: SPL_KVS_SPREAD 2 (readers over two pools as well) vs 1, mixed step
set -x
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r2_91
mkdir -p $O
B="--host-api 0 --embed-e2e 0"
for o in 2 1 2 1; do SPL_KVS_SPREAD=$o timeout -k 10 200 python bench.py $B | sed "s/^{/{\"spread\": $o, /" >> $O/mixed.jsonl 2>> $O/mixed.err || exit 1; done &&
echo done
