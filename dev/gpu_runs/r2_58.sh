# round 2, call 58: per-call ring latency breakdown (stamps variant: device segments + shader clock), 1 and 16 threads
set -x
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r2_58
mkdir -p $O
B=libsplinter_amd/bin/splinter_hostapi_bench
SPLINTER_HIP_LIB=$PWD/libsplinter_amd/lib/libsplinter_hip_stamps.so timeout -k 10 60 $B --store hbm:st1 --threads 1 --seconds 2 > $O/t1.jsonl 2>&1 &&
SPLINTER_HIP_LIB=$PWD/libsplinter_amd/lib/libsplinter_hip_stamps.so timeout -k 10 60 $B --store hbm:st16 --threads 16 --seconds 2 > $O/t16.jsonl 2>&1 &&

echo done
