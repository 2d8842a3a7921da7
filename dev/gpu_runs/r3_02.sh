# round 3, call 2: residual+LN kernel pipeline / epilogue variants (numerics + A/B)
set -x
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r3_02
mkdir -p $O
for v in 10 11 20 21 30 31; do NOMIC_RLN=$v timeout -k 10 120 python -u -m pytest tests/test_nomic_gpu.py -x -q --timeout 60 --timeout-method thread -k "residual_layernorm" > $O/pytest_v$v.log 2>&1 || exit 1; done
timeout -k 10 300 python scripts/residual_gemm_ab.py --rln-variants 10,11,20,21,30,31 > $O/rln_ab.jsonl 2> $O/rln_ab.err &&
echo done
