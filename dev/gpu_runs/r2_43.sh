# round 2, call 42: ring v3: tickets spread over the worker waves
set -x
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r2_43
mkdir -p $O
T=libsplinter_amd/bin/splinter_hostapi_bench
timeout -k 10 200 python -u -m pytest tests/test_ring_gpu.py -x -v --timeout 150 --timeout-method thread > $O/ring_tests.log 2>&1 &&
for th in 1 4 16 32; do timeout -k 10 60 $T --store hbm:hb$th --threads $th --seconds 2 --keys 65536 --value-len 150 >> $O/hostapi.jsonl 2>> $O/hostapi.err || exit 1; done &&
echo done
