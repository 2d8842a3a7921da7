# round 3, call 8: decoder prefill-over-cache attention (hd 64/128), Q8G32 weights, node-store TAP;
# EPI2/PF2 residual variants; bench.py with the search arena, routed N=1 row and query phase
set -x
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r3_08
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_splainference.py tests/test_node_gpu.py -x -v -m gpu --timeout 120 --timeout-method thread > $O/pytest_dec_node.log 2>&1 || exit 1
for v in 1222 2222 3222; do NOMIC_RLN=$v timeout -k 10 120 python -u -m pytest tests/test_nomic_gpu.py -x -q --timeout 60 --timeout-method thread -k "residual_layernorm" > $O/pytest_v$v.log 2>&1 || exit 1; done
timeout -k 10 300 python scripts/residual_gemm_ab.py --rln-variants 222,1222,2222,3222 > $O/rln_ab.jsonl 2> $O/rln_ab.err || exit 1
timeout -k 10 300 python bench.py --keys-per-gpu 10000000 --search-keys 2000000 --steps 5 --warmup 2 --embed-e2e 3 > $O/bench_small.json 2> $O/bench_small.err || exit 1
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > $O/bench_default.json 2> $O/bench_default.err || exit 1
echo done
