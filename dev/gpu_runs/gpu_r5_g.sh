#!/bin/bash
set -o pipefail
OUT=gpurun_out/r5g
mkdir -p $OUT
export TMPDIR=/tmp


timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_embed -o run -- python3 bench.py --mode embed --steps 5 --warmup 2 --embed-e2e 0 --host-api 0 --host-api-threads2 0 --search-keys 0 --daemon-docs 0 --exchange-ab 0 --mixed5 0 > $OUT/embed.out 2> $OUT/embed.err || { tail -20 $OUT/embed.err; exit 1; }
f=$(find $OUT/prof_embed -name '*kernel_stats.csv' | head -1); head -14 "$f" | cut -c1-200
