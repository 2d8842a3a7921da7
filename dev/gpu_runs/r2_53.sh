# round 2, call 53: residual projections on hipBLASLt in the encoder -- numerics + embed / mixed A/B
set -x
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r2_53
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_nomic_gpu.py -x -v --timeout 240 --timeout-method thread -k "encoder" > $O/tests.log 2>&1 &&
for b in 1 0 1 0; do NOMIC_RESIDUAL_BLAS=$b timeout -k 10 200 python bench.py --mode embed --host-api 0 --embed-e2e 0 | sed "s/^{/{\"residual_blas\": $b, /" >> $O/embed.jsonl 2>> $O/embed.err || exit 1; done &&
for b in 1 0; do NOMIC_RESIDUAL_BLAS=$b timeout -k 10 200 python bench.py --host-api 0 --embed-e2e 0 | sed "s/^{/{\"residual_blas\": $b, /" >> $O/mixed.jsonl 2>> $O/mixed.err || exit 1; done &&
echo done
