# round 2, call 99: q4 GEMV with 8 rows per wave (SPL_Q4_ROWS=8) -- numerics under the knob and decode A/B
set -x
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r2_99
mkdir -p $O
SPL_Q4_ROWS=8 timeout -k 10 300 python -u -m pytest tests/test_splainference.py -x -v --timeout 200 --timeout-method thread -m gpu -k "q4" > $O/tests.log 2>&1 &&
for r in 8 4; do SPL_Q4_ROWS=$r timeout -k 10 400 python -u scripts/decode_q4_bench.py --layers 8 | sed "s/^{/{\"rows\": $r, /" >> $O/decode.jsonl 2>> $O/decode.err || exit 1; done &&
echo done
