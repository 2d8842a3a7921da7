#!/bin/bash
# Residual+LN kernel forms on one MI355X: their GPU tests, the per-shape A/B (o-proj, down) and
# bench.py --mode embed per form (alternating), then the default mixed bench per form.
set -o pipefail
OUT=${OUT:-gpurun_out/rln}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_nomic_gpu.py -m gpu -k "row_complete" -x -v --timeout 150 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -3 $OUT/tests.log
timeout -k 10 300 python -u scripts/residual_gemm_ab.py --no-blas --rln-variants 222,232 --rounds 7 > $OUT/ab.out 2> $OUT/ab.err || { tail -20 $OUT/ab.err; exit 1; }
grep us_median $OUT/ab.out
for v in 222 232 222 232; do NOMIC_RLN=$v timeout -k 10 300 python -u bench.py --mode embed --steps 20 --warmup 5 > $OUT/embed_$v.out 2>/dev/null || exit 1; python3 -c "import json,sys; d=json.loads(open('$OUT/embed_$v.out').read().strip().splitlines()[-1]); print('$v', d['ms_per_step'], d.get('embed_vectors_per_s'))"; done
for v in 222 232; do NOMIC_RLN=$v timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $OUT/bench_$v.out 2>/dev/null || exit 1; python3 -c "import json,sys; d=json.loads(open('$OUT/bench_$v.out').read().strip().splitlines()[-1]); print('mixed $v', d['ms_per_step'], d['value'])"; done
