set -x
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_gpu18.log 2>&1 &&
timeout -k 10 300 python scripts/kv_micro.py --batch 8000000 > gpurun_out/kv18.log 2>&1 &&
SPLINTER_ARENA_UGET=4 timeout -k 10 300 python scripts/kv_micro.py --batch 8000000 > gpurun_out/kv18_g4.log 2>&1 &&
timeout -k 10 400 python bench.py --mode kv > gpurun_out/bench18_kv.log 2>&1 &&
timeout -k 10 400 python bench.py > gpurun_out/bench18.log 2>&1 &&
echo done
