# round 2, call 94: tokenizer worker pool vs a thread per worker per batch (SPL_TOK_POOL), e2e embedding A/B
set -x
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r2_94
mkdir -p $O
B="--mode embed --host-api 0 --steps 3 --warmup 1 --keys-per-gpu 1000000 --embed-e2e 40"
for o in 1 0 1 0 1 0; do SPL_TOK_POOL=$o timeout -k 10 200 python bench.py $B | sed "s/^{/{\"pool\": $o, /" >> $O/e2e.jsonl 2>> $O/e2e.err || exit 1; done &&
echo done
