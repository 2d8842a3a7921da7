# decode-attention kernel: numerics vs fp32, decoder GPU tests, SDPA vs kernel per-token latency
set -x
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_splainference.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_dec66.log 2>&1 &&
timeout -k 10 300 python scripts/decode_bench.py > gpurun_out/decode66.log 2>&1 &&
timeout -k 10 300 python scripts/decode_bench.py --kv-heads 2 --prefill 1900 --steps 100 >> gpurun_out/decode66.log 2>&1 &&
echo done
