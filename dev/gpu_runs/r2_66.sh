# round 2, call 66: zero-copy raw_ptr on hbm: stores (dmabuf host mapping); ring / arena / search tests
set -x
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r2_66
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_ring_gpu.py tests/test_arena_gpu.py tests/test_search_gpu.py -x -v --timeout 200 --timeout-method thread > $O/tests.log 2>&1 &&
echo done
