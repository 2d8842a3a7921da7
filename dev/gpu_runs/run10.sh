# full GPU suite, default bench (serial KV then embed), kv-only bench, default-bench kernel profile
set -x
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_gpu10.log 2>&1 &&
timeout -k 10 400 python bench.py > gpurun_out/bench10.log 2>&1 &&
timeout -k 10 400 python bench.py --mode kv > gpurun_out/bench10_kv.log 2>&1 &&
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof10 -o bench --output-format csv -- python3 bench.py --steps 5 --warmup 2 > gpurun_out/prof10.log 2>&1 &&
echo done
