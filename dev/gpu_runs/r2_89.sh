# round 2, call 89: decoder prefill with is_causal SDPA for head dim 128
set -x
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r2_89
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_splainference.py -x -v --timeout 200 --timeout-method thread -m gpu > $O/tests.log 2>&1 &&
echo done
