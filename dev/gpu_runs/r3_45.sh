# round 3, call 45: persistent 256^2 GEMM with asm LDS-DMA (NOMIC_GEMM=515) -- numerics, bitwise race screen vs
# the builtin-DMA persistent kernel, GEMM A/B against the peeled launch-per-tile default
set -x
cd $GRAFT_REPO_ROOT
O=gpurun_out/r3_45
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_nomic_gpu.py -x -v -m gpu --timeout 150 --timeout-method thread -k "gemm" > $O/pytest_gemm.log 2>&1 || exit 1
timeout -k 10 300 python -u scripts/gemm_race_screen.py --runs 20 --knob variant --value 515 > $O/race.jsonl 2> $O/race.err || exit 1
timeout -k 10 300 python -u scripts/gemm_bench.py --variants 256,512,515 --pps 2 --sregs 0 --shapes ffn_swiglu,qkv_rope --rounds 9 > $O/gemm_ab.jsonl 2> $O/gemm_ab.err || exit 1
echo done
