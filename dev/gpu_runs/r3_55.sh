# round 3, call 55: short-cache decode attention widened to 16 waves (8 for 8 heads per KV head), key groups
# reduced by shuffles then LDS -- decode tests with it on, per-token A/B
set -x
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r3_55
mkdir -p $O
SPL_DEC_SMALL=1 timeout -k 10 400 python -u -m pytest tests/test_splainference.py -x -v -m gpu --timeout 150 --timeout-method thread > $O/pytest_dec.log 2>&1 || exit 1
for sm in 1 0 1 0; do
  SPL_DEC_SMALL=$sm timeout -k 10 300 python -u scripts/decode_q4_bench.py --layers 8 --rounds 2 2>> $O/d.err | sed "s/^{/{\"small\": $sm, /" >> $O/dec.jsonl || exit 1
done
SPL_DEC_SMALL=1 timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/dec -o dec -- python3 scripts/decode_q4_bench.py --layers 8 --rounds 2 > $O/decp.json 2> $O/decp.err || exit 1
find $O -name "*kernel_trace.csv" -delete
echo done
