#!/bin/bash
# arena / route GPU tests on the current tree (server claim-section change)
set -o pipefail
OUT=gpurun_out/r6s17
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_arena_gpu.py tests/test_route_gpu.py -x -v --timeout 300 --timeout-method thread > $OUT/tests.txt 2>&1
rc=$?; tail -3 $OUT/tests.txt; grep -cE "PASSED" $OUT/tests.txt; exit $rc
