#!/bin/bash
# per-call ring: timed sleep-polls vs futex waiting (SPLINTER_RING_WAIT=futex), CPU per call
set -o pipefail
OUT=gpurun_out/r5z
mkdir -p $OUT
H=./libsplinter_amd/bin/splinter_hostapi_bench
timeout -k 10 600 python -u -m pytest tests/test_ring_gpu.py -x -v --timeout 150 --timeout-method thread > $OUT/ring_tests.txt 2>&1 || { tail -30 $OUT/ring_tests.txt; exit 1; }
tail -2 $OUT/ring_tests.txt
for rep in 1 2; do
  for w in sleep futex; do
    for t in 1 16 32 64 128; do
      SPLINTER_RING_WAIT=$w timeout -k 10 120 $H --store hbm:rz$t$w --threads $t --seconds 2 --keys 20000 \
        > $OUT/t${t}_$w.$rep.out 2> $OUT/t${t}_$w.$rep.err || { tail -5 $OUT/t${t}_$w.$rep.err; exit 1; }
      echo "$w t$t: $(cat $OUT/t${t}_$w.$rep.out)"
    done
    SPLINTER_RING_WAIT=$w timeout -k 10 120 $H --store hbm:rzp$w --procs 4 --threads 16 --seconds 2 --keys 20000 \
      > $OUT/p4t16_$w.$rep.out 2> $OUT/p4t16_$w.$rep.err || { tail -5 $OUT/p4t16_$w.$rep.err; exit 1; }
    echo "$w p4t16: $(cat $OUT/p4t16_$w.$rep.out)"
  done
done
