# round 2, call 60: ring v3 default (single doorbell read): full GPU suite, host-API sweep
set -x
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r2_60
mkdir -p $O
T=libsplinter_amd/bin/splinter_hostapi_bench
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 &&
for th in 1 4 8 16 24 32; do timeout -k 10 60 $T --store hbm:v3$th --threads $th --seconds 2 --keys 65536 --value-len 150 >> $O/hostapi.jsonl 2>> $O/hostapi.err || exit 1; done &&
echo done
