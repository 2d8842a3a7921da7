# round 3, call 26: software-pipelined cooperative row copy (SPLINTER_ARENA_PIPE=1/2) -- arena tests,
# KV-only and get-only A/B (acquire-free get on in all rows)
set -x
cd $GRAFT_REPO_ROOT
O=gpurun_out/r3_26
mkdir -p $O
export SPLINTER_ARENA_COOP_GET=2
SPLINTER_ARENA_PIPE=1 timeout -k 10 300 python -u -m pytest tests/test_arena_gpu.py -x -v -m gpu --timeout 120 --timeout-method thread > $O/pytest_arena_pipe1.log 2>&1 || exit 1
SPLINTER_ARENA_PIPE=2 timeout -k 10 300 python -u -m pytest tests/test_arena_gpu.py -x -v -m gpu --timeout 120 --timeout-method thread > $O/pytest_arena_pipe2.log 2>&1 || exit 1
K="--mode kv --host-api 0 --host-api-threads2 0 --routed-steps 0 --steps 10 --warmup 2"
run() { tag=$1; shift; e=(); while [[ $1 == *=* ]]; do e+=("$1"); shift; done; env "${e[@]}" timeout -k 10 300 python -u bench.py $K "$@" 2>> $O/kv.err | sed "s/^{/{\"tag\": \"$tag\", /" >> $O/kv_ab.jsonl; }
for r in 1 2; do
run base SPLINTER_ARENA_PIPE=0 || exit 1
run pipe1 SPLINTER_ARENA_PIPE=1 || exit 1
run pipe2 SPLINTER_ARENA_PIPE=2 || exit 1
done
for p in 0 1 2; do run get_only_p$p SPLINTER_ARENA_PIPE=$p --set-frac 0.0 || exit 1; run set_only_p$p SPLINTER_ARENA_PIPE=$p --set-frac 1.0 || exit 1; done
echo done
