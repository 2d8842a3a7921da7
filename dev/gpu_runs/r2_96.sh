# round 2, call 96: hipBLASLt residual GEMMs on M rounded up to 256 for varlen batches (NOMIC_BLAS_PAD) -- tests + e2e A/B
set -x
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r2_96
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_nomic_gpu.py tests/test_search_gpu.py -x -v --timeout 200 --timeout-method thread -m gpu > $O/tests.log 2>&1 &&
B="--mode embed --host-api 0 --steps 3 --warmup 1 --keys-per-gpu 1000000 --embed-e2e 40"
for o in 1 0 1 0; do NOMIC_BLAS_PAD=$o timeout -k 10 200 python bench.py $B | sed "s/^{/{\"pad\": $o, /" >> $O/e2e.jsonl 2>> $O/e2e.err || exit 1; done &&
echo done
