# round 2, call 56: splinference batched hbm path
set -x
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r2_56
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_search_gpu.py -x -v --timeout 300 --timeout-method thread -k "splinference" > $O/tests.log 2>&1 &&
echo done
