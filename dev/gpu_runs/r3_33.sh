# round 3, call 33: register SwiGLU epilogue of the launch-per-tile 256^2 GEMM (k_gemm256 EPI 1) --
# numerics, GEMM A/B on the encoder's SwiGLU shape, embed-only bench with it on / off
set -x
cd $GRAFT_REPO_ROOT
O=gpurun_out/r3_33
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_nomic_gpu.py -x -v -m gpu --timeout 150 --timeout-method thread -k "swiglu or encoder" > $O/pytest_swiglu.log 2>&1 || exit 1
timeout -k 10 200 python -u scripts/gemm_bench.py --variants 256 --sregs 0,1 --shapes ffn_swiglu --rounds 9 > $O/gemm_ab.jsonl 2> $O/gemm_ab.err || exit 1
E="--mode embed --embed-e2e 0 --daemon-docs 0 --host-api 0 --host-api-threads2 0 --routed-steps 0 --steps 20 --warmup 5"
run() { tag=$1; shift; e=(); while [[ $1 == *=* ]]; do e+=("$1"); shift; done; env "${e[@]}" timeout -k 10 300 python -u bench.py "$@" 2>> $O/b.err | sed "s/^{/{\"tag\": \"$tag\", /" >> $O/ab.jsonl; }
for r in 1 2; do
run embed_sreg0 NOMIC_SWIGLU_REG=0 $E || exit 1
run embed_sreg1 NOMIC_SWIGLU_REG=1 $E || exit 1
done
echo done
