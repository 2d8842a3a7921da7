# round 3, call 42: residual+LN kernel with the K steps rotated per block (NOMIC_RLN=20222): numerics, time vs K,
# embed A/B
set -x
cd $GRAFT_REPO_ROOT
O=gpurun_out/r3_42
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_nomic_gpu.py -x -v -m gpu --timeout 150 --timeout-method thread -k "residual_layernorm" > $O/pytest_rln.log 2>&1 || exit 1
timeout -k 10 300 python -u scripts/residual_gemm_ab.py --no-blas --rln-variants 222,20222 --ks 128,768,3072 > $O/rln_k.jsonl 2> $O/rln_k.err || exit 1
E="--mode embed --embed-e2e 0 --daemon-docs 0 --host-api 0 --host-api-threads2 0 --routed-steps 0 --steps 20 --warmup 5"
run() { tag=$1; shift; e=(); while [[ $1 == *=* ]]; do e+=("$1"); shift; done; env "${e[@]}" timeout -k 10 300 python -u bench.py "$@" 2>> $O/b.err | sed "s/^{/{\"tag\": \"$tag\", /" >> $O/ab.jsonl; }
for r in 1 2; do
run embed_222 NOMIC_RLN=222 $E || exit 1
run embed_rot NOMIC_RLN=20222 $E || exit 1
done
echo done
