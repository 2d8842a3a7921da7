# round 2, call 41: bench with the end-to-end embed measurement, embed-only, full GPU suite, smoke
set -x
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r2_41
mkdir -p $O
timeout -k 10 300 python bench.py > $O/mixed.json 2> $O/mixed.err &&
timeout -k 10 200 python bench.py --mode embed --host-api 0 > $O/embed.json 2> $O/embed.err &&
timeout -k 10 800 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 &&
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 &&
echo done
