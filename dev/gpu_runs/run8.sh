# GEMM 256 numerics + A/B microbench, then bench with per-priority streams
set -x
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_nomic_gpu.py -q -x > gpurun_out/pytest_nomic8.log 2>&1 &&
timeout -k 10 300 python scripts/gemm_bench.py --tokens 32768 > gpurun_out/gemm8_32k.log 2>&1 &&
timeout -k 10 300 python scripts/gemm_bench.py --tokens 262144 --rounds 3 --iters 3 > gpurun_out/gemm8_256k.log 2>&1 &&
timeout -k 10 400 python bench.py --steps 10 --warmup 3 > gpurun_out/bench8.log 2>&1 &&
timeout -k 10 400 python bench.py --mode embed --steps 5 --warmup 2 --embed-batch 512 > gpurun_out/bench8_embed.log 2>&1 &&
echo done
