# round 3, call 47: get-kernel shape with the acquire-free get now default: 1 op per lane, 512-thread blocks
set -x
cd $GRAFT_REPO_ROOT
O=gpurun_out/r3_47
mkdir -p $O
SPLINTER_ARENA_UGET=1 timeout -k 10 300 python -u -m pytest tests/test_arena_gpu.py -x -v -m gpu --timeout 120 --timeout-method thread > $O/pytest_arena_uget1.log 2>&1 || exit 1
K="--mode kv --host-api 0 --host-api-threads2 0 --routed-steps 0 --steps 10 --warmup 2"
run() { tag=$1; shift; e=(); while [[ $1 == *=* ]]; do e+=("$1"); shift; done; env "${e[@]}" timeout -k 10 300 python -u bench.py "$@" 2>> $O/b.err | sed "s/^{/{\"tag\": \"$tag\", /" >> $O/ab.jsonl; }
for r in 1 2; do
run kv_base X=1 $K || exit 1
run kv_uget1 SPLINTER_ARENA_UGET=1 $K || exit 1
run kv_bget512 SPLINTER_ARENA_BLOCK_GET=512 $K || exit 1
run kv_uget4 SPLINTER_ARENA_UGET=4 $K || exit 1
done
echo done
