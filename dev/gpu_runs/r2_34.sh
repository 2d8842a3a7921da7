# round 2, call 34: VMM vs hipMalloc arena (KV + mixed), the whole GPU suite, smoke
set -x
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r2_34
mkdir -p $O
timeout -k 10 200 python bench.py --mode kv --host-api 0 > $O/kv_vmm.json 2> $O/kv_vmm.err &&
SPLINTER_HBM_VMM=0 timeout -k 10 200 python bench.py --mode kv --host-api 0 > $O/kv_malloc.json 2> $O/kv_malloc.err &&
timeout -k 10 200 python bench.py > $O/mixed.json 2> $O/mixed.err &&
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 &&
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 &&
echo done
