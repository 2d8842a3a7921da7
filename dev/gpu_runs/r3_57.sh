# round 3, call 57: the grouped decode-attention kernel as the split form for long caches (splits of <= 512 keys,
# k_attn_combine as before) -- decode tests, per-token A/B at a 3000-token prompt and at the short cache
set -x
cd $GRAFT_REPO_ROOT
O=gpurun_out/r3_57
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_splainference.py -x -v -m gpu --timeout 150 --timeout-method thread > $O/pytest_dec.log 2>&1 || exit 1
for sm in 1 0 1 0; do
  SPL_DEC_SMALL=$sm timeout -k 10 300 python -u scripts/decode_q4_bench.py --layers 8 --rounds 2 --prompt 3000 2>> $O/d.err | sed "s/^{/{\"small\": $sm, \"prompt\": 3000, /" >> $O/dec.jsonl || exit 1
done
SPL_DEC_SMALL=1 timeout -k 10 300 python -u scripts/decode_q4_bench.py --layers 8 --rounds 2 2>> $O/d.err | sed "s/^{/{\"small\": 1, \"prompt\": 128, /" >> $O/dec.jsonl || exit 1
echo done
