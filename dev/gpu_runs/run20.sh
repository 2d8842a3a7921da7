set -x
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_gpu20.log 2>&1 &&
timeout -k 10 300 python scripts/kv_micro.py --batch 8000000 > gpurun_out/kv20.log 2>&1 &&
timeout -k 10 400 python bench.py > gpurun_out/bench20.log 2>&1 &&
echo done
