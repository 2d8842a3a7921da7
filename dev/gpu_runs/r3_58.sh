# round 3, call 58: software-pipelined row copy in the (acquire-free, 2-op) get kernel (SPLINTER_ARENA_PIPE=2)
# with the session-2 defaults, KV-only and mixed, alternating
set -x
cd $GRAFT_REPO_ROOT
O=gpurun_out/r3_58
mkdir -p $O
SPLINTER_ARENA_PIPE=2 timeout -k 10 300 python -u -m pytest tests/test_arena_gpu.py -x -v -m gpu --timeout 120 --timeout-method thread > $O/pytest_arena_pipe2.log 2>&1 || exit 1
K="--mode kv --host-api 0 --host-api-threads2 0 --routed-steps 0 --steps 10 --warmup 2"
M="--mode mixed --embed-e2e 0 --daemon-docs 0 --search-batches 2 --host-api 0 --host-api-threads2 0 --routed-steps 0 --steps 20 --warmup 5"
run() { tag=$1; shift; e=(); while [[ $1 == *=* ]]; do e+=("$1"); shift; done; env "${e[@]}" timeout -k 10 300 python -u bench.py "$@" 2>> $O/b.err | sed "s/^{/{\"tag\": \"$tag\", /" >> $O/ab.jsonl; }
for r in 1 2; do
run kv_base X=1 $K || exit 1
run kv_pipe2 SPLINTER_ARENA_PIPE=2 $K || exit 1
run mixed_base X=1 $M || exit 1
run mixed_pipe2 SPLINTER_ARENA_PIPE=2 $M || exit 1
done
echo done
