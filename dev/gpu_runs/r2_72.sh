# round 2, call 72: 4-bit (Q4G32) decode weights -- numerics tests, decoder GPU suite, bf16 vs q4 per-token A/B
set -x
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r2_72
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_splainference.py -x -v --timeout 200 --timeout-method thread -m gpu > $O/tests.log 2>&1 &&
timeout -k 10 400 python -u scripts/decode_q4_bench.py --layers 8 > $O/decode_q4.jsonl 2> $O/decode_q4.err &&
echo done
