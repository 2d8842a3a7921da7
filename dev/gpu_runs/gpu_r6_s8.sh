#!/bin/bash
# maintenance pass on its low-priority stream beside queued KV steps; then the s6 attribution runs
set -o pipefail
OUT=gpurun_out/r6s8
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_maint_gpu.py -k "online_beside" -v -s --timeout 300 --timeout-method thread > $OUT/maint.txt 2>&1
rc=$?; grep -E "PASSED|FAILED|^E " $OUT/maint.txt | cut -c1-300 | tail -10; grep -o "overlapped_steps[^r]*" $OUT/maint.txt; grep -o "dead_status[^l]*" $OUT/maint.txt
[ $rc -le 1 ] || exit 1
bash dev/gpu_runs/gpu_r6_s6.sh
