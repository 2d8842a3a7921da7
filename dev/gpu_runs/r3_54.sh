# round 3, call 54: grouped three-phase decode attention for caches <= 512 keys (k_attn_decode_g) -- decode
# numerics (all head dims / group sizes, device-side lengths), decode engine tests, per-token A/B
set -x
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r3_54
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_splainference.py -x -v -m gpu --timeout 150 --timeout-method thread > $O/pytest_dec.log 2>&1 || exit 1
for sm in 1 0 1 0; do
  SPL_DEC_SMALL=$sm timeout -k 10 300 python -u scripts/decode_q4_bench.py --layers 8 --rounds 2 2>> $O/d.err | sed "s/^{/{\"small\": $sm, /" >> $O/dec.jsonl || exit 1
done
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/dec -o dec -- python3 scripts/decode_q4_bench.py --layers 8 --rounds 2 > $O/decp.json 2> $O/decp.err || exit 1
find $O -name "*kernel_trace.csv" -delete
echo done
