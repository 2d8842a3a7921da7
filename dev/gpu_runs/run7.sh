# full GPU test suite + bench sweeps (steps chained: stop at the first failure)
set -x
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_gpu7.log 2>&1 &&
timeout -k 10 400 python bench.py --steps 10 --warmup 3 > gpurun_out/bench7.log 2>&1 &&
timeout -k 10 400 python bench.py --mode kv --steps 10 --warmup 3 > gpurun_out/bench7_kv.log 2>&1 &&
timeout -k 10 400 python bench.py --embed-batch 32 --steps 10 --warmup 3 > gpurun_out/bench7_e32.log 2>&1 &&
timeout -k 10 400 python bench.py --embed-batch 128 --steps 10 --warmup 3 > gpurun_out/bench7_e128.log 2>&1 &&
echo done
