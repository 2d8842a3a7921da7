set -x
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1200 python -m pytest tests/test_bench_gpu.py -q -x > gpurun_out/pytest_bench15.log 2>&1
echo rc=$?
