# round 2, call 55: update claim without the post-CAS re-check round trip -- arena integrity tests, then KV / mixed A/B vs the re-check build
set -x
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r2_55
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_arena_gpu.py tests/test_ring_gpu.py tests/test_route_gpu.py -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 &&
for v in "" recheck "" recheck; do SPLINTER_HIP_VARIANT=$v timeout -k 10 200 python bench.py --mode kv --host-api 0 --embed-e2e 0 | sed "s/^{/{\"variant\": \"$v\", /" >> $O/kv.jsonl 2>> $O/kv.err || exit 1; done &&
for v in "" recheck; do SPLINTER_HIP_VARIANT=$v timeout -k 10 200 python bench.py --host-api 0 --embed-e2e 0 | sed "s/^{/{\"variant\": \"$v\", /" >> $O/mixed.jsonl 2>> $O/mixed.err || exit 1; done &&
echo done
