# round 2, call 27: new GPU tests (CLI search on the device, dequant parity) + full suite
set -x
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r2_27
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_search_gpu.py tests/test_nomic_gpu.py -x -v -s --timeout 300 --timeout-method thread > $O/pytest_new.log 2>&1 &&
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 &&
echo done
