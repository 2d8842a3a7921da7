# round 3, call 49: software-pipelined attention (k_attn4, variant 17: QK^T of tile t+1 beside the softmax of
# tile t) -- varlen numerics, attention A/B against k_attn3, embed A/B
set -x
cd $GRAFT_REPO_ROOT
O=gpurun_out/r3_49
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_nomic_gpu.py -x -v -m gpu --timeout 150 --timeout-method thread -k "attention_varlen" > $O/pytest_attn.log 2>&1 || exit 1
ATTN_VARIANTS=13,17 timeout -k 10 200 python -u scripts/attn_bench.py --rounds 7 > $O/attn_ab.jsonl 2> $O/attn_ab.err || exit 1
E="--mode embed --embed-e2e 0 --daemon-docs 0 --host-api 0 --host-api-threads2 0 --routed-steps 0 --steps 20 --warmup 5"
run() { tag=$1; shift; e=(); while [[ $1 == *=* ]]; do e+=("$1"); shift; done; env "${e[@]}" timeout -k 10 300 python -u bench.py "$@" 2>> $O/b.err | sed "s/^{/{\"tag\": \"$tag\", /" >> $O/ab.jsonl; }
for r in 1 2; do
run embed_a13 NOMIC_ATTN=13 $E || exit 1
run embed_a17 NOMIC_ATTN=17 $E || exit 1
done
echo done
