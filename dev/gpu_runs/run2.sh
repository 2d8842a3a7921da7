set -x
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -q > gpurun_out/pytest_gpu2.log 2>&1
echo "pytest rc=$?"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_kv -o kv --output-format csv -- python3 bench.py --steps 5 --warmup 2 > gpurun_out/bench_prof.log 2>&1
echo "prof rc=$?"
