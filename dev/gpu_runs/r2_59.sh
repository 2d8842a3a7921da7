# round 2, call 59: ring v3 (host key hash, overlapped header loads, register payloads, pipelined
# doorbell polls): ring GPU tests, then host-API latency A/B (v3 vs v3 with one poll in flight)
set -x
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r2_59
mkdir -p $O
B=libsplinter_amd/bin/splinter_hostapi_bench
L=$PWD/libsplinter_amd/lib
timeout -k 10 300 python -u -m pytest tests/test_ring_gpu.py -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1 &&
for t in 1 16; do
  timeout -k 10 60 $B --store hbm:a$t --threads $t --seconds 2 > $O/v3_t$t.jsonl 2>&1 || exit 1
  SPLINTER_HIP_LIB=$L/libsplinter_hip_poll1.so timeout -k 10 60 $B --store hbm:b$t --threads $t --seconds 2 > $O/poll1_t$t.jsonl 2>&1 || exit 1
  SPLINTER_HIP_LIB=$L/libsplinter_hip_stamps.so timeout -k 10 60 $B --store hbm:c$t --threads $t --seconds 2 > $O/stamps_t$t.jsonl 2>&1 || exit 1
done
for t in 1 16; do
  timeout -k 10 60 $B --store hbm:d$t --threads $t --seconds 2 > $O/v3b_t$t.jsonl 2>&1 || exit 1
  SPLINTER_HIP_LIB=$L/libsplinter_hip_poll1.so timeout -k 10 60 $B --store hbm:e$t --threads $t --seconds 2 > $O/poll1b_t$t.jsonl 2>&1 || exit 1
done
echo done
