# round 3, call 6: residual as an identity-MFMA K step (EPI 2) and 2-pair W prefetch (PF 2)
set -x
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r3_06
mkdir -p $O
for v in 1222 2222 3222; do NOMIC_RLN=$v timeout -k 10 120 python -u -m pytest tests/test_nomic_gpu.py -x -q --timeout 60 --timeout-method thread -k "residual_layernorm" > $O/pytest_v$v.log 2>&1 || exit 1; done
timeout -k 10 300 python scripts/residual_gemm_ab.py --rln-variants 222,1222,2222,3222 > $O/rln_ab.jsonl 2> $O/rln_ab.err || exit 1
echo done
