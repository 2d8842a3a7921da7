# round 3, call 51: sets at ONE op per lane on the carried-retry kernel (SPLINTER_ARENA_U=1: 4x the workgroups of
# the round-2 dispatch) -- arena tests, KV-only and mixed A/B; decode per-kernel profile (splainference)
set -x
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r3_51
mkdir -p $O
SPLINTER_ARENA_U=1 timeout -k 10 300 python -u -m pytest tests/test_arena_gpu.py tests/test_route_gpu.py -x -v -m gpu --timeout 120 --timeout-method thread > $O/pytest_u1.log 2>&1 || exit 1
K="--mode kv --host-api 0 --host-api-threads2 0 --routed-steps 0 --steps 10 --warmup 2"
M="--mode mixed --embed-e2e 0 --daemon-docs 0 --search-batches 2 --host-api 0 --host-api-threads2 0 --routed-steps 0 --steps 20 --warmup 5"
run() { tag=$1; shift; e=(); while [[ $1 == *=* ]]; do e+=("$1"); shift; done; env "${e[@]}" timeout -k 10 300 python -u bench.py "$@" 2>> $O/b.err | sed "s/^{/{\"tag\": \"$tag\", /" >> $O/ab.jsonl; }
for r in 1 2; do
run kv_u2 X=1 $K || exit 1
run kv_u1 SPLINTER_ARENA_U=1 $K || exit 1
run mixed_u2 X=1 $M || exit 1
run mixed_u1 SPLINTER_ARENA_U=1 $M || exit 1
done
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/dec -o dec -- python3 scripts/decode_q4_bench.py --layers 8 --rounds 2 > $O/dec.json 2> $O/dec.err || exit 1
find $O -name "*kernel_trace.csv" -delete
echo done
