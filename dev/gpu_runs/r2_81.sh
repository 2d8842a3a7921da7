# round 2, call 81: split count sweep of the split-L decode attention (SPL_DEC_SPLITS) at llama-7B head shapes
set -x
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r2_81
mkdir -p $O
for sp in 0 4 8 16 32; do
  if [ $sp = 0 ]; then unset SPL_DEC_SPLITS; else export SPL_DEC_SPLITS=$sp; fi
  timeout -k 10 200 python -u scripts/attn_decode_micro.py --attn-only | sed "s/^{/{\"splits\": $sp, /" >> $O/sweep.jsonl 2>> $O/sweep.err || exit 1
done
echo done
