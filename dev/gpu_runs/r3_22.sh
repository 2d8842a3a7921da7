# round 3, call 22: write-through cooperative set kernel (SPLINTER_ARENA_COOP=2: sc1 row stores, no
# per-round L2 write-back) -- arena tests under it, KV-only and mixed A/B against the release form
set -x
cd $GRAFT_REPO_ROOT
O=gpurun_out/r3_22
mkdir -p $O
SPLINTER_ARENA_COOP=2 timeout -k 10 300 python -u -m pytest tests/test_arena_gpu.py -x -v -m gpu --timeout 120 --timeout-method thread > $O/pytest_arena_coop2.log 2>&1 || exit 1
K="--mode kv --host-api 0 --host-api-threads2 0 --routed-steps 0 --steps 10 --warmup 2"
for v in 1 2 1 2; do SPLINTER_ARENA_COOP=$v timeout -k 10 300 python -u bench.py $K 2>> $O/kv.err | sed "s/^{/{\"coop\": $v, /" >> $O/kv_ab.jsonl || exit 1; done
M="--host-api 0 --host-api-threads2 0 --routed-steps 0 --embed-e2e 0 --daemon-docs 0 --search-batches 2 --steps 20 --warmup 5"
for v in 1 2; do SPLINTER_ARENA_COOP=$v timeout -k 10 400 python -u bench.py $M 2>> $O/mixed.err | sed "s/^{/{\"coop\": $v, /" >> $O/mixed_ab.jsonl || exit 1; done
echo done
