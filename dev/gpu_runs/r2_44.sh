# round 2, call 44: ring with 32 worker waves (spread tickets), 1/4/8/16/24 host threads
set -x
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r2_44
mkdir -p $O
T=libsplinter_amd/bin/splinter_hostapi_bench
timeout -k 10 200 python -u -m pytest tests/test_ring_gpu.py -x -v --timeout 150 --timeout-method thread > $O/ring_tests.log 2>&1 &&
for sp in 1; do for th in 1 4 8 16 24 32; do SPLINTER_RING_SPREAD=$sp timeout -k 10 60 $T --store hbm:hb$sp$th --threads $th --seconds 2 --keys 65536 --value-len 150 | sed "s/^{/{\"spread\": $sp, /" >> $O/hostapi.jsonl 2>> $O/hostapi.err || exit 1; done; done &&
echo done
