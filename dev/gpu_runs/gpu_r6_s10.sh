#!/bin/bash
# per-call floor (stamps in device memory after the completion); concurrent-maintenance overlap
# report; the GPU suite and the default bench on the current tree
set -o pipefail
OUT=gpurun_out/r6s10
mkdir -p $OUT
STAMPS=$PWD/libsplinter_amd/lib/libsplinter_hip_stamps.so
for t in 1 16 32; do
  SPLINTER_HIP_LIB=$STAMPS timeout -k 10 120 libsplinter_amd/bin/splinter_hostapi_bench --store hbm:stamp$t --threads $t --seconds 3 --keys 65536 --value-len 150 > $OUT/stamps_t$t.out 2> $OUT/stamps_t$t.err || { tail -5 $OUT/stamps_t$t.err; exit 1; }
  echo "t=$t"; cat $OUT/stamps_t$t.out; head -8 $OUT/stamps_t$t.err
done
for t in 1 16 32; do
  timeout -k 10 120 libsplinter_amd/bin/splinter_hostapi_bench --store hbm:nost$t --threads $t --seconds 3 --keys 65536 --value-len 150 > $OUT/nostamps_t$t.out 2> $OUT/nostamps_t$t.err || exit 1
  echo "default t=$t"; cat $OUT/nostamps_t$t.out
done
timeout -k 10 600 python -u -m pytest tests/test_maint_gpu.py -k "online_beside" -v -s --timeout 300 --timeout-method thread > $OUT/maint.txt 2>&1
rc=$?; grep -E "PASSED|FAILED|^E " $OUT/maint.txt | cut -c1-300 | tail -6; grep -o "overlapped_steps[^r]*" $OUT/maint.txt; grep -o "dead_status[^l]*" $OUT/maint.txt
[ $rc -le 1 ] || exit 1
timeout -k 10 1200 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.txt 2>&1; echo "suite rc=$?"
tail -6 $OUT/pytest_gpu.txt
timeout -k 10 900 python -u bench.py > $OUT/bench.out 2> $OUT/bench.err || { tail -30 $OUT/bench.err; exit 1; }
tail -c 3500 $OUT/bench.out
