#!/bin/bash
# online maintenance v2 (phase-2 reclaim sweep), search C ABI changes, then the GPU suite + bench
set -o pipefail
OUT=gpurun_out/r6maint2
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_maint_gpu.py tests/test_search_gpu.py tests/test_arena_gpu.py tests/test_node_gpu.py tests/test_ring_gpu.py -x -v -s --timeout 300 --timeout-method thread > $OUT/maint_tests.txt 2>&1 || { grep -E "PASS|FAIL|Error|assert" $OUT/maint_tests.txt | tail -40; exit 1; }
grep -E "PASSED|FAILED|'rehash'" $OUT/maint_tests.txt | tail -40
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.txt 2>&1 || { tail -40 $OUT/pytest_gpu.txt; exit 1; }
tail -3 $OUT/pytest_gpu.txt
timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 --embed-e2e 0 --host-api 0 --host-api-threads2 0 --daemon-docs 0 --exchange-ab 0 --mixed5 0 > $OUT/bench.out 2> $OUT/bench.err || { tail -30 $OUT/bench.err; exit 1; }
tail -c 2500 $OUT/bench.out
