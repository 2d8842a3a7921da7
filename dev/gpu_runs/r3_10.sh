# round 3, call 10: decoder / node / ring GPU tests; GEMM DMA-interleave (ILV) numerics + A/B;
# late-load attention variants; residual+LN variants; bench.py (search arena, routed N=1, query phase)
set -x
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r3_10
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_splainference.py tests/test_node_gpu.py tests/test_ring_gpu.py -x -v -m gpu --timeout 150 --timeout-method thread > $O/pytest_dec_node_ring.log 2>&1 || exit 1
timeout -k 10 400 python -u -m pytest tests/test_nomic_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread -k "gemm_store or asymmetric or swiglu_and_rope or attention_varlen" > $O/pytest_gemm_attn.log 2>&1 || exit 1
timeout -k 10 300 python -u scripts/gemm_bench.py --variants 512,256,128 --ilvs 0,1,2 --shapes qkv_rope,ffn_swiglu --rounds 5 > $O/gemm_ilv_ab.jsonl 2> $O/gemm_ilv_ab.err || exit 1
ATTN_VARIANTS=6,10,7,11,9,12 timeout -k 10 200 python -u scripts/attn_bench.py > $O/attn_ab.jsonl 2> $O/attn_ab.err || exit 1
for v in 1222 2222 3222; do NOMIC_RLN=$v timeout -k 10 120 python -u -m pytest tests/test_nomic_gpu.py -x -q --timeout 60 --timeout-method thread -k "residual_layernorm" > $O/pytest_v$v.log 2>&1 || exit 1; done
timeout -k 10 300 python scripts/residual_gemm_ab.py --rln-variants 222,1222,2222,3222 > $O/rln_ab.jsonl 2> $O/rln_ab.err || exit 1
timeout -k 10 300 python bench.py --keys-per-gpu 10000000 --search-keys 2000000 --steps 5 --warmup 2 --embed-e2e 3 > $O/bench_small.json 2> $O/bench_small.err || exit 1
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > $O/bench_default.json 2> $O/bench_default.err || exit 1
echo done
