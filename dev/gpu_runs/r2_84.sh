# round 2, call 84: GQA-shared split-L decode attention (one workgroup per kv group and split)
set -x
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r2_84
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_splainference.py -x -v --timeout 200 --timeout-method thread -m gpu > $O/tests.log 2>&1 &&
timeout -k 10 300 python -u scripts/attn_decode_micro.py --attn-only > $O/micro.jsonl 2> $O/micro.err &&
timeout -k 10 400 python -u scripts/decode_q4_bench.py --layers 8 --prompt 3000 > $O/decode_q4_ctx3000.jsonl 2> $O/decode_q4_ctx3000.err &&
echo done
