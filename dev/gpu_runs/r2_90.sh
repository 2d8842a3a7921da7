# round 2, call 90: writer slices over two hardware-queue pools (SPL_KVS_SPREAD) A/B, mixed and KV-only
set -x
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r2_90
mkdir -p $O
B="--host-api 0 --embed-e2e 0"
for o in 1 0 1 0; do SPL_KVS_SPREAD=$o timeout -k 10 200 python bench.py $B | sed "s/^{/{\"spread\": $o, /" >> $O/mixed.jsonl 2>> $O/mixed.err || exit 1; done &&
for o in 1 0; do SPL_KVS_SPREAD=$o timeout -k 10 200 python bench.py --mode kv $B | sed "s/^{/{\"spread\": $o, /" >> $O/kv.jsonl 2>> $O/kv.err || exit 1; done &&
echo done
