# round 2, call 50: attention ILV variant (per-q-block S / softmax / PV order) -- numerics + A/B
set -x
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r2_50
mkdir -p $O
timeout -k 10 200 python -u -m pytest tests/test_nomic_gpu.py -x -v --timeout 150 --timeout-method thread -k "attention_varlen" > $O/tests.log 2>&1 &&
ATTN_VARIANTS=6,7,8,6,7 timeout -k 10 200 python scripts/attn_bench.py --rounds 7 > $O/attn_ab.jsonl 2> $O/attn_ab.err &&
echo done
