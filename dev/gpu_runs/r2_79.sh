# round 2, call 79: e2e pipeline on one stream (fetch enqueued ahead of the encoder) -- mixed (default) and embed-only benches
set -x
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r2_79
mkdir -p $O
timeout -k 10 300 python bench.py --host-api 0 --embed-e2e 20 > $O/mixed.json 2> $O/mixed.err &&
timeout -k 10 200 python bench.py --mode embed --host-api 0 --embed-e2e 20 --steps 10 --keys-per-gpu 1000000 > $O/embed.json 2> $O/embed.err &&
timeout -k 10 300 python -u -m pytest tests/test_search_gpu.py -x -v --timeout 200 --timeout-method thread -m gpu > $O/tests.log 2>&1 &&
echo done
