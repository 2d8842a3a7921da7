set -x
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu1.log 2>&1
echo "pytest rc=$?"
timeout -k 10 300 python bench.py --keys-per-gpu 10000000 --batch 4000000 --steps 5 --warmup 2 > gpurun_out/bench_small.log 2>&1
echo "bench small rc=$?"
timeout -k 10 400 python bench.py --steps 5 --warmup 2 > gpurun_out/bench_full.log 2>&1
echo "bench full rc=$?"
