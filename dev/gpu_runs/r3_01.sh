# round 3, call 1: row-complete residual+LN kernel — numerics, A/B vs split and hipBLASLt, embed-only bench
set -x
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r3_01
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_nomic_gpu.py -x -v --timeout 120 --timeout-method thread -k "residual_layernorm or encoder_matches or shipped_shape" > $O/pytest_rln.log 2>&1 &&
timeout -k 10 200 python scripts/residual_gemm_ab.py > $O/rln_ab.jsonl 2> $O/rln_ab.err &&
timeout -k 10 200 python bench.py --mode embed --steps 20 --warmup 3 > $O/bench_embed_fused.json 2> $O/bench_embed_fused.err &&
NOMIC_SCHEDULE=split timeout -k 10 200 python bench.py --mode embed --steps 20 --warmup 3 > $O/bench_embed_split.json 2> $O/bench_embed_split.err &&
echo done
