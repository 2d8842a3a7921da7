# round 2, call 52: residual projections -- fused MFMA epilogue vs hipBLASLt beta=1 in place
set -x
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r2_52
mkdir -p $O
timeout -k 10 200 python scripts/residual_gemm_ab.py > $O/ab.jsonl 2> $O/ab.err &&
echo done
