# round 2, call 28: CLI search on the device (progress printed)
set -x
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r2_28
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_search_gpu.py -x -v -s -k cli_search --timeout 240 --timeout-method thread 2>&1 | tee $O/pytest_cli.log
