# round 3, call 20: k_attn3 as the default attention (encoder / attention tests), 4-wave variant A/B,
# persistent-GEMM relaxed epilogue A/B (512 vs 256), embed bench + default bench
set -x
cd $GRAFT_REPO_ROOT
O=gpurun_out/r3_20
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_nomic_gpu.py -x -v -m gpu --timeout 150 --timeout-method thread > $O/pytest_nomic.log 2>&1 || exit 1
ATTN_VARIANTS=13,16 timeout -k 10 200 python -u scripts/attn_bench.py --rounds 7 > $O/attn_ab.jsonl 2> $O/attn_ab.err || exit 1
timeout -k 10 300 python -u scripts/gemm_bench.py --variants 512,256 --ilvs 0,1 --shapes ffn_swiglu,qkv_rope > $O/gemm_ab.jsonl 2> $O/gemm_ab.err || exit 1
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || exit 1
echo done
