set -x
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_search_gpu.py -q > gpurun_out/pytest_search6.log 2>&1; echo "pytest rc=$?"
timeout -k 10 600 python bench.py --steps 10 --warmup 3 > gpurun_out/bench6.log 2>&1; echo "bench rc=$?"
timeout -k 10 600 python bench.py --mode embed --steps 5 --warmup 2 > gpurun_out/bench6_embed.log 2>&1; echo "bench embed rc=$?"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof6 -o mixed --output-format csv -- python3 bench.py --steps 5 --warmup 2 > gpurun_out/bench6_prof.log 2>&1; echo "prof rc=$?"
echo done
