# attention v2 numerics + A/B, GEMM auto selection, embed-mode profile
set -x
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_nomic_gpu.py -q -x > gpurun_out/pytest_nomic9.log 2>&1 &&
timeout -k 10 300 python scripts/attn_bench.py --docs 64 > gpurun_out/attn9_64.log 2>&1 &&
timeout -k 10 300 python scripts/attn_bench.py --docs 512 --rounds 3 --iters 3 > gpurun_out/attn9_512.log 2>&1 &&
timeout -k 10 400 python bench.py --mode embed --steps 5 --warmup 2 --embed-batch 512 > gpurun_out/bench9_embed.log 2>&1 &&
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof9 -o embed --output-format csv -- python3 bench.py --mode embed --steps 3 --warmup 1 --embed-batch 512 --keys-per-gpu 1000000 > gpurun_out/prof9.log 2>&1 &&
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof9 -o mixed --output-format csv -- python3 bench.py --steps 3 --warmup 1 > gpurun_out/prof9m.log 2>&1 &&
echo done
