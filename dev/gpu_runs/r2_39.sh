# round 2, call 39: stream-K persistent GEMM (variant 514) -- numerics, then per-shape A/B vs the other kernels + hipBLASLt
set -x
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r2_39
mkdir -p $O
timeout -k 10 200 python -u -m pytest tests/test_nomic_gpu.py -x -v --timeout 150 --timeout-method thread -k "stream_k or store_and_residual or swiglu_and_rope" > $O/tests.log 2>&1 &&
timeout -k 10 300 python scripts/gemm_bench.py --rounds 7 > $O/gemm_ab.jsonl 2> $O/gemm_ab.err &&
echo done
