#!/bin/bash
# online maintenance (seqlocked moves beside live traffic), mode-3 acquire + timeout statuses: the
# new tests first, then the whole GPU suite and the bench (the KV path carries the maintenance seq)
set -o pipefail
OUT=gpurun_out/r6maint
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_maint_gpu.py tests/test_arena_gpu.py -x -v -s --timeout 240 --timeout-method thread > $OUT/maint_tests.txt 2>&1 || { tail -60 $OUT/maint_tests.txt; exit 1; }
grep -E "PASS|FAIL|rehash=|dead_status" $OUT/maint_tests.txt | tail -30
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.txt 2>&1 || { tail -40 $OUT/pytest_gpu.txt; exit 1; }
tail -3 $OUT/pytest_gpu.txt
timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 --embed-e2e 0 --host-api 0 --host-api-threads2 0 --daemon-docs 0 --exchange-ab 0 --mixed5 0 --search-keys 0 > $OUT/bench.out 2> $OUT/bench.err || { tail -30 $OUT/bench.err; exit 1; }
tail -c 1500 $OUT/bench.out
