#!/bin/bash
# attention: MFMA row sum + max3 chains (variant 16) vs k_attn3 (13): numerics tests, kernel A/B, encoder A/B
set -o pipefail
OUT=gpurun_out/r5j
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_nomic_gpu.py -k "attention or full_encoder" > $OUT/tests.txt 2>&1 || { tail -30 $OUT/tests.txt; exit 1; }
tail -3 $OUT/tests.txt
ATTN_VARIANTS=13,16 timeout -k 10 300 python scripts/attn_bench.py --rounds 7 > $OUT/attn_ab.jsonl 2> $OUT/attn_ab.err || { tail -20 $OUT/attn_ab.err; exit 1; }
cat $OUT/attn_ab.jsonl
for v in 13 16 13 16; do
  NOMIC_ATTN=$v timeout -k 10 300 python bench.py --mode embed --steps 20 --warmup 5 > $OUT/embed_$v.out 2> $OUT/embed_$v.err || { tail -20 $OUT/embed_$v.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('$OUT/embed_$v.out').read().strip().splitlines()[-1]); print($v, d['ms_per_step'], d['embed_phase_ms_per_step'])"
done
