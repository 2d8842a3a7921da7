# round 2, call 64: 8-wave 256-row attention blocks (variant 9) numerics + A/B against variant 6
set -x
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r2_64
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_nomic_gpu.py -x -v --timeout 120 --timeout-method thread -k "attention_varlen" > $O/tests.log 2>&1 &&
ATTN_VARIANTS=6,9 timeout -k 10 300 python -u scripts/attn_bench.py --rounds 7 > $O/attn.jsonl 2>&1 &&
echo done
