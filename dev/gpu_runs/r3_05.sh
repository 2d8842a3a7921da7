# round 3, call 5: interleave density / A-ring depth variants of the residual+LN kernel
set -x
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r3_05
mkdir -p $O
for v in 212 222 213 242 243; do NOMIC_RLN=$v timeout -k 10 120 python -u -m pytest tests/test_nomic_gpu.py -x -q --timeout 60 --timeout-method thread -k "residual_layernorm" > $O/pytest_v$v.log 2>&1 || exit 1; done
timeout -k 10 300 python scripts/residual_gemm_ab.py --rln-variants 220,212,222,213,242,243 > $O/rln_ab.jsonl 2> $O/rln_ab.err || exit 1
echo done
