# round 3, call 27: set publication by an 8-B store instead of the epoch-increment atomic
# (SPLINTER_ARENA_FINISH_STORE=1) -- arena tests, KV-only / set-only A/B
set -x
cd $GRAFT_REPO_ROOT
O=gpurun_out/r3_27
mkdir -p $O
export SPLINTER_ARENA_COOP_GET=2
SPLINTER_ARENA_FINISH_STORE=1 timeout -k 10 300 python -u -m pytest tests/test_arena_gpu.py -x -v -m gpu --timeout 120 --timeout-method thread > $O/pytest_arena_fs.log 2>&1 || exit 1
K="--mode kv --host-api 0 --host-api-threads2 0 --routed-steps 0 --steps 10 --warmup 2"
run() { tag=$1; shift; e=(); while [[ $1 == *=* ]]; do e+=("$1"); shift; done; env "${e[@]}" timeout -k 10 300 python -u bench.py $K "$@" 2>> $O/kv.err | sed "s/^{/{\"tag\": \"$tag\", /" >> $O/kv_ab.jsonl; }
for r in 1 2; do
run base SPLINTER_ARENA_FINISH_STORE=0 || exit 1
run fs SPLINTER_ARENA_FINISH_STORE=1 || exit 1
run set_only_base SPLINTER_ARENA_FINISH_STORE=0 --set-frac 1.0 || exit 1
run set_only_fs SPLINTER_ARENA_FINISH_STORE=1 --set-frac 1.0 || exit 1
done
echo done
