#!/bin/bash
# ring fixes + the reworked bench JSON (timed-output integrity, exchange A/B, mixed5)
set -o pipefail
OUT=gpurun_out/r5b
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_ring_gpu.py -x -v --timeout 120 --timeout-method thread > $OUT/ring.txt 2>&1 || { tail -40 $OUT/ring.txt; exit 1; }
tail -3 $OUT/ring.txt
timeout -k 10 700 python bench.py --steps 20 --warmup 5 > $OUT/bench.out 2> $OUT/bench.err || { tail -30 $OUT/bench.err; exit 1; }
tail -1 $OUT/bench.out
grep -E "exchange|integrity" $OUT/bench.err | tail -8
