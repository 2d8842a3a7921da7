# round 2, call 76: sampler with replicated histogram bins; decode attention / sampler microbenchmarks
set -x
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r2_76
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_splainference.py -x -v --timeout 200 --timeout-method thread -m gpu -k "sample or attn_decode or engine" > $O/tests.log 2>&1 &&
timeout -k 10 300 python -u scripts/attn_decode_micro.py > $O/micro.jsonl 2> $O/micro.err &&
echo done
