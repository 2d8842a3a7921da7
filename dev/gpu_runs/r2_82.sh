# round 2, call 82: multi-block sampler chain (dec_sample_ws) -- tests, microbenchmark, 8-layer decode
set -x
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r2_82
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_splainference.py -x -v --timeout 200 --timeout-method thread -m gpu > $O/tests.log 2>&1 &&
timeout -k 10 300 python -u scripts/attn_decode_micro.py > $O/micro.jsonl 2> $O/micro.err &&
timeout -k 10 400 python -u scripts/decode_q4_bench.py --layers 8 > $O/decode_q4.jsonl 2> $O/decode_q4.err &&
echo done
