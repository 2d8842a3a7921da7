# round 3, call 52: decode attention at short caches -- the single-workgroup kernel (default below 512 keys)
# against the GQA split kernel forced to 2 / 4 / 8 splits (SPL_DEC_SPLITS), per-token latency
set -x
cd $GRAFT_REPO_ROOT
O=gpurun_out/r3_52
mkdir -p $O
for sp in 0 2 4 8; do
  if [ $sp = 0 ]; then e=X=1; else e=SPL_DEC_SPLITS=$sp; fi
  env $e timeout -k 10 300 python -u scripts/decode_q4_bench.py --layers 8 --rounds 2 2>> $O/d.err | sed "s/^{/{\"splits\": $sp, /" >> $O/dec.jsonl || exit 1
done
echo done
