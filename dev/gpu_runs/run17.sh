set -x
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_nomic_gpu.py -q -x > gpurun_out/pytest_nomic17.log 2>&1 &&
timeout -k 10 300 python scripts/gemm_bench.py --tokens 32768 > gpurun_out/gemm17_32k.log 2>&1 &&
timeout -k 10 300 python scripts/gemm_bench.py --tokens 262144 --rounds 3 --iters 3 > gpurun_out/gemm17_256k.log 2>&1 &&
echo done
