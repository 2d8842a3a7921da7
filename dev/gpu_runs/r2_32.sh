# round 2, call 32: VMM-chunk arenas -- attach time vs size, cross-process tests, KV bench A/B
set -x
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r2_32
mkdir -p $O
for n in 262144 1000000 4000000; do timeout -k 10 120 python -u scripts/ipc_open_debug.py $n >> $O/ipc.log 2>&1 || exit 1; done
timeout -k 10 300 python -u -m pytest tests/test_arena_gpu.py tests/test_ring_gpu.py -x -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 &&
timeout -k 10 200 python bench.py --mode kv --host-api 0 > $O/kv_vmm.json 2> $O/kv_vmm.err &&
SPLINTER_HBM_VMM=0 timeout -k 10 200 python bench.py --mode kv --host-api 0 > $O/kv_malloc.json 2> $O/kv_malloc.err &&
echo done
