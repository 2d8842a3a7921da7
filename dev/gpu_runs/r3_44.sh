# round 3, call 44: KV fan-out with the writers on the high-priority queue pool (SPL_KVS_PRIO=1), KV-only and mixed,
# alternating with the default
set -x
cd $GRAFT_REPO_ROOT
O=gpurun_out/r3_44
mkdir -p $O
K="--mode kv --host-api 0 --host-api-threads2 0 --routed-steps 0 --steps 10 --warmup 2"
M="--mode mixed --embed-e2e 0 --daemon-docs 0 --search-batches 2 --host-api 0 --host-api-threads2 0 --routed-steps 0 --steps 20 --warmup 5"
run() { tag=$1; shift; e=(); while [[ $1 == *=* ]]; do e+=("$1"); shift; done; env "${e[@]}" timeout -k 10 300 python -u bench.py "$@" 2>> $O/b.err | sed "s/^{/{\"tag\": \"$tag\", /" >> $O/ab.jsonl; }
for r in 1 2; do
run kv_base X=1 $K || exit 1
run kv_wprio SPL_KVS_PRIO=1 $K || exit 1
run mixed_base X=1 $M || exit 1
run mixed_wprio SPL_KVS_PRIO=1 $M || exit 1
done
echo done
