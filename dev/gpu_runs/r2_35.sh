# round 2, call 35: new GPU tests (12-layer encoder vs fp32 at 64x512, cross-process reader race), then the suite
set -x
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r2_35
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_nomic_gpu.py tests/test_arena_gpu.py -x -v --timeout 300 --timeout-method thread -k "twelve or full or cross_process_reader" > $O/new_tests.log 2>&1 &&
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 &&
echo done
