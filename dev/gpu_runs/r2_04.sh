# round 2, call 4: command-ring per-call API (new GPU tests + host-API numbers at 1..32 threads),
# then the whole GPU suite
set -x
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r2_04
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_ring_gpu.py -x -v -s --timeout 120 --timeout-method thread > $O/pytest_ring.log 2>&1 &&
for t in 1 4 16 32; do timeout -k 10 60 ./libsplinter_amd/bin/splinter_hostapi_bench --store hbm:hapi$t --threads $t --seconds 2 --keys 65536 --append-check 8 > $O/hostapi_t$t.json 2> $O/hostapi_t$t.err || exit 1; done &&
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 &&
echo done
