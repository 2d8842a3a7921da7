# round 3, call 32: new KV defaults (U=2 sets, acquire-free gets) -- arena/ring/route/node GPU tests;
# overlapped KV + embed phases on the native fan-out (--overlap-native 1) vs serial, alternating
set -x
cd $GRAFT_REPO_ROOT
O=gpurun_out/r3_32
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_arena_gpu.py tests/test_ring_gpu.py tests/test_route_gpu.py tests/test_node_gpu.py -x -v -m gpu --timeout 150 --timeout-method thread > $O/pytest_kv.log 2>&1 || exit 1
M="--mode mixed --embed-e2e 0 --daemon-docs 0 --search-batches 2 --host-api 0 --host-api-threads2 0 --routed-steps 0 --steps 20 --warmup 5"
run() { tag=$1; shift; e=(); while [[ $1 == *=* ]]; do e+=("$1"); shift; done; env "${e[@]}" timeout -k 10 300 python -u bench.py "$@" 2>> $O/b.err | sed "s/^{/{\"tag\": \"$tag\", /" >> $O/ab.jsonl; }
for r in 1 2; do
run serial X=1 $M || exit 1
run overlap X=1 $M --overlap-native 1 || exit 1
run overlap_nothrottle X=1 $M --overlap-native 1 --throttle 0 || exit 1
done
echo done
