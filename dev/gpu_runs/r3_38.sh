# round 3, call 38: asm LDS-DMA (counted lgkmcnt) in the residual+LN kernel (NOMIC_RLN=1xxxx) and the 128^2
# GEMM (NOMIC_GEMM_AS128); PP=2 now the 256^2 default -- numerics, bitwise race screens, A/Bs
set -x
cd $GRAFT_REPO_ROOT
O=gpurun_out/r3_38
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_nomic_gpu.py -x -v -m gpu --timeout 150 --timeout-method thread -k "gemm or encoder" > $O/pytest_gemm.log 2>&1 || exit 1
timeout -k 10 200 python -u scripts/gemm_race_screen.py --runs 20 --knob rln --value 10222 > $O/race_rln.jsonl 2> $O/race.err || exit 1
timeout -k 10 200 python -u scripts/gemm_race_screen.py --runs 20 --knob rln --value 12222 >> $O/race_rln.jsonl 2>> $O/race.err || exit 1
timeout -k 10 200 python -u scripts/gemm_race_screen.py --runs 20 --knob as128 --value 1 > $O/race_as128.jsonl 2>> $O/race.err || exit 1
timeout -k 10 300 python -u scripts/residual_gemm_ab.py --no-blas --rln-variants 222,10222,12222,10220,10020 > $O/rln_ab.jsonl 2> $O/rln_ab.err || exit 1
timeout -k 10 300 python -u scripts/gemm_bench.py --variants 128,256 --pps 2 --as128 0,1 --sregs 0 --shapes qkv_rope --rounds 9 > $O/gemm_ab.jsonl 2> $O/gemm_ab.err || exit 1
E="--mode embed --embed-e2e 0 --daemon-docs 0 --host-api 0 --host-api-threads2 0 --routed-steps 0 --steps 20 --warmup 5"
run() { tag=$1; shift; e=(); while [[ $1 == *=* ]]; do e+=("$1"); shift; done; env "${e[@]}" timeout -k 10 300 python -u bench.py "$@" 2>> $O/b.err | sed "s/^{/{\"tag\": \"$tag\", /" >> $O/ab.jsonl; }
for r in 1 2; do
run embed_base X=1 $E || exit 1
run embed_rlnasm NOMIC_RLN=10222 $E || exit 1
run embed_rlnasm_as128 NOMIC_RLN=10222 NOMIC_GEMM_AS128=1 $E || exit 1
done
echo done
