# round 3, call 37: peeled lockstep 256^2 GEMM with asm LDS-DMA (NOMIC_GEMM_PP=2: counted lgkmcnt before
# the MFMAs instead of lgkmcnt(0)) -- numerics, bitwise race screen, GEMM A/B, embed A/B
set -x
cd $GRAFT_REPO_ROOT
O=gpurun_out/r3_37
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_nomic_gpu.py -x -v -m gpu --timeout 150 --timeout-method thread -k "gemm" > $O/pytest_gemm.log 2>&1 || exit 1
timeout -k 10 300 python -u scripts/gemm_race_screen.py --runs 30 --value 2 > $O/race.jsonl 2> $O/race.err || exit 1
timeout -k 10 300 python -u scripts/gemm_bench.py --variants 256 --pps 0,2 --sregs 0,1 --shapes ffn_swiglu,qkv_rope --rounds 9 > $O/gemm_ab.jsonl 2> $O/gemm_ab.err || exit 1
E="--mode embed --embed-e2e 0 --daemon-docs 0 --host-api 0 --host-api-threads2 0 --routed-steps 0 --steps 20 --warmup 5"
run() { tag=$1; shift; e=(); while [[ $1 == *=* ]]; do e+=("$1"); shift; done; env "${e[@]}" timeout -k 10 300 python -u bench.py "$@" 2>> $O/b.err | sed "s/^{/{\"tag\": \"$tag\", /" >> $O/ab.jsonl; }
for r in 1 2; do
run embed_pp0 NOMIC_GEMM_PP=0 $E || exit 1
run embed_pp2 NOMIC_GEMM_PP=2 $E || exit 1
done
echo done
