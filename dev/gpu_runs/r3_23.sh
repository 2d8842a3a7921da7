# round 3, call 23: acquire-free get kernel (SPLINTER_ARENA_COOP_GET=2) and 16-B-key (KW4) coop
# kernels -- arena tests under them, KV-only A/B
set -x
cd $GRAFT_REPO_ROOT
O=gpurun_out/r3_23
mkdir -p $O
SPLINTER_ARENA_COOP_GET=2 timeout -k 10 300 python -u -m pytest tests/test_arena_gpu.py -x -v -m gpu --timeout 120 --timeout-method thread > $O/pytest_arena_get2.log 2>&1 || exit 1
SPLINTER_ARENA_COOP_GET=2 SPLINTER_ARENA_KW4=1 timeout -k 10 300 python -u -m pytest tests/test_arena_gpu.py -x -v -m gpu --timeout 120 --timeout-method thread > $O/pytest_arena_get2_kw4.log 2>&1 || exit 1
K="--mode kv --host-api 0 --host-api-threads2 0 --routed-steps 0 --steps 10 --warmup 2"
run() { tag=$1; shift; env "$@" timeout -k 10 300 python -u bench.py $K 2>> $O/kv.err | sed "s/^{/{\"tag\": \"$tag\", /" >> $O/kv_ab.jsonl; }
for r in 1 2; do
run base SPLINTER_ARENA_COOP_GET=1 || exit 1
run get2 SPLINTER_ARENA_COOP_GET=2 || exit 1
run get2_kw4 SPLINTER_ARENA_COOP_GET=2 SPLINTER_ARENA_KW4=1 || exit 1
done
echo done
