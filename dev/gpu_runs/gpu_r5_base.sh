#!/bin/bash
# round-5 baseline on a fresh box: GPU suite, embed-only and the default bench
set -o pipefail
OUT=gpurun_out/r5a
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.txt 2>&1 || { tail -30 $OUT/pytest_gpu.txt; exit 1; }
tail -3 $OUT/pytest_gpu.txt
timeout -k 10 300 python bench.py --mode embed --steps 10 --warmup 3 --embed-e2e 0 --host-api 0 --host-api-threads2 0 --search-keys 0 --daemon-docs 0 --routed-steps 0 > $OUT/embed.out 2> $OUT/embed.err || { tail -20 $OUT/embed.err; exit 1; }
tail -1 $OUT/embed.out
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $OUT/bench.out 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
tail -1 $OUT/bench.out
