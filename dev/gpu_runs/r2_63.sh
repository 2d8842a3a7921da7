# round 2, call 63: ring v3 final default (host key hash, overlapped header loads, register set
# payloads, staged get): hbm-store GPU tests, host-API sweep, latency breakdown
set -x
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r2_63
mkdir -p $O
T=libsplinter_amd/bin/splinter_hostapi_bench
L=$PWD/libsplinter_amd/lib
timeout -k 10 400 python -u -m pytest tests/test_ring_gpu.py tests/test_arena_gpu.py tests/test_search_gpu.py -x -v --timeout 200 --timeout-method thread > $O/tests.log 2>&1 &&
for th in 1 4 8 16 24 32; do timeout -k 10 60 $T --store hbm:f$th --threads $th --seconds 2 --keys 65536 --value-len 150 >> $O/hostapi.jsonl 2>> $O/hostapi.err || exit 1; done &&
SPLINTER_HIP_LIB=$L/libsplinter_hip_stamps.so timeout -k 10 60 $T --store hbm:s1 --threads 1 --seconds 2 --keys 65536 --value-len 150 > $O/stamps_t1.jsonl 2>&1 &&
SPLINTER_HIP_LIB=$L/libsplinter_hip_stamps.so timeout -k 10 60 $T --store hbm:s16 --threads 16 --seconds 2 --keys 65536 --value-len 150 > $O/stamps_t16.jsonl 2>&1 &&
timeout -k 10 60 $T --store hbm:ap --threads 8 --seconds 1 --keys 4096 --value-len 150 --append-check 64 > $O/append.jsonl 2>&1 &&
echo done
