# round 2, call 93: e2e embedding with the pooled tokenizer -- embed-only and default mixed bench
set -x
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r2_93
mkdir -p $O
timeout -k 10 200 python bench.py --mode embed --host-api 0 --steps 10 --keys-per-gpu 1000000 > $O/embed.json 2> $O/embed.err &&
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err &&
timeout -k 10 300 python -u -m pytest tests/test_search_gpu.py tests/test_nomic_gpu.py -x -v --timeout 200 --timeout-method thread -m gpu > $O/tests.log 2>&1 &&
echo done
