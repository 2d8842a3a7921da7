# round 2, call 71: spl_kvs_step submission order A/B (interleaved writer/reader slices vs writers first)
set -x
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r2_71
mkdir -p $O
B="--host-api 0 --embed-e2e 0"
for o in 1 0 1 0; do SPL_KVS_ORDER=$o timeout -k 10 200 python bench.py $B | sed "s/^{/{\"kvs_order\": $o, /" >> $O/mixed.jsonl 2>> $O/mixed.err || exit 1; done &&
for o in 1 0; do SPL_KVS_ORDER=$o timeout -k 10 200 python bench.py --mode kv $B | sed "s/^{/{\"kvs_order\": $o, /" >> $O/kv.jsonl 2>> $O/kv.err || exit 1; done &&
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/prof -o run -- python3 bench.py --steps 10 --warmup 2 $B > $O/bench_prof.json 2> $O/bench_prof.err &&
echo done
