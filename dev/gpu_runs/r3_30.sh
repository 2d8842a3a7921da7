# round 3, call 30 (re-run of the lost call 28): is the KV step bound by hardware-queue
# serialisation?  ops per lane (more workgroups per dispatch) and hardware queues per priority,
# KV-only and mixed
set -x
cd $GRAFT_REPO_ROOT
O=gpurun_out/r3_30
mkdir -p $O
K="--mode kv --host-api 0 --host-api-threads2 0 --routed-steps 0 --steps 10 --warmup 2"
run() { tag=$1; shift; e=(); while [[ $1 == *=* ]]; do e+=("$1"); shift; done; env "${e[@]}" timeout -k 10 300 python -u bench.py $K "$@" 2>> $O/kv.err | sed "s/^{/{\"tag\": \"$tag\", /" >> $O/kv_ab.jsonl; }
run base X=1 || exit 1
run u2 SPLINTER_ARENA_U=2 || exit 1
run u1 SPLINTER_ARENA_U=1 SPLINTER_ARENA_UGET=1 || exit 1
run uget1 SPLINTER_ARENA_UGET=1 || exit 1
run u2_uget1 SPLINTER_ARENA_U=2 SPLINTER_ARENA_UGET=1 || exit 1
run hwq4 SPLINTER_BENCH_HW_QUEUES=4 || exit 1
run hwq8 SPLINTER_BENCH_HW_QUEUES=8 || exit 1
run ws8 X=1 --writer-streams 8 --reader-streams 8 || exit 1
run base X=1 || exit 1
M="--mode mixed --embed-e2e 0 --daemon-docs 0 --search-batches 2 --steps 20 --warmup 5"
run mixed_base X=1 $M || exit 1
run mixed_u2_uget1 SPLINTER_ARENA_U=2 SPLINTER_ARENA_UGET=1 $M || exit 1
run mixed_hwq4 SPLINTER_BENCH_HW_QUEUES=4 $M || exit 1
echo done
