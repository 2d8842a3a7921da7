# round-end verification from a fresh rebuild: GPU suite, smoke, default bench, kernel stats
set -x
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu64.log 2>&1 &&
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke64.log 2>&1 &&
timeout -k 10 400 python bench.py > gpurun_out/bench64.log 2>&1 &&
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof64 -o bench --output-format csv -- python3 bench.py --steps 5 --warmup 2 > gpurun_out/prof64.log 2>&1 &&
echo done
