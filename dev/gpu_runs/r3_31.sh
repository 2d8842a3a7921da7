# round 3, call 31: sets at 2 ops per lane (SPLINTER_ARENA_U=2: twice the workgroups per set
# dispatch) in the KV-only and mixed steps, alternating with the default; with the acquire-free get
set -x
cd $GRAFT_REPO_ROOT
O=gpurun_out/r3_31
mkdir -p $O
SPLINTER_ARENA_U=2 timeout -k 10 300 python -u -m pytest tests/test_arena_gpu.py -x -v -m gpu --timeout 120 --timeout-method thread > $O/pytest_arena_u2.log 2>&1 || exit 1
K="--mode kv --host-api 0 --host-api-threads2 0 --routed-steps 0 --steps 10 --warmup 2"
M="--mode mixed --embed-e2e 0 --daemon-docs 0 --search-batches 2 --host-api 0 --host-api-threads2 0 --routed-steps 0 --steps 20 --warmup 5"
run() { tag=$1; shift; e=(); while [[ $1 == *=* ]]; do e+=("$1"); shift; done; env "${e[@]}" timeout -k 10 300 python -u bench.py "$@" 2>> $O/kv.err | sed "s/^{/{\"tag\": \"$tag\", /" >> $O/kv_ab.jsonl; }
for r in 1 2; do
run mixed_base X=1 $M || exit 1
run mixed_u2 SPLINTER_ARENA_U=2 $M || exit 1
run mixed_u2_get2 SPLINTER_ARENA_U=2 SPLINTER_ARENA_COOP_GET=2 $M || exit 1
done
run kv_u2 SPLINTER_ARENA_U=2 $K || exit 1
run kv_u2_get2 SPLINTER_ARENA_U=2 SPLINTER_ARENA_COOP_GET=2 $K || exit 1
run kv_u2_b512 SPLINTER_ARENA_U=2 SPLINTER_ARENA_BLOCK=512 $K || exit 1
run kv_u2_ws16 SPLINTER_ARENA_U=2 $K --writer-streams 16 --reader-streams 16 || exit 1
run kv_u2_set SPLINTER_ARENA_U=2 $K --set-frac 1.0 || exit 1
run kv_u2 SPLINTER_ARENA_U=2 $K || exit 1
echo done
