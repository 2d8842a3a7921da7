# round 2, call 74: histogram nucleus search in dec_sample, q4 GEMV with early/prefetched weight loads
set -x
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r2_74
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_splainference.py -x -v --timeout 200 --timeout-method thread -m gpu > $O/tests.log 2>&1 &&
timeout -k 10 400 python -u scripts/decode_q4_bench.py --layers 8 > $O/decode_q4.jsonl 2> $O/decode_q4.err &&
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/prof -o run -- python3 scripts/decode_q4_bench.py --layers 2 --tokens 16 --rounds 1 > $O/dq4.jsonl 2> $O/dq4.err &&
echo done
