#!/bin/bash
# KV step modes x fused-grid schedules (spl_kvs_set_sched) against the plain kernels
set -o pipefail
OUT=gpurun_out/r6s28
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_arena_gpu.py -v -k "kvs" --timeout 300 --timeout-method thread > $OUT/tests.txt 2>&1
rc=$?; grep -E "PASSED|FAILED|ERROR" $OUT/tests.txt | cut -c1-120; tail -1 $OUT/tests.txt; exit $rc
