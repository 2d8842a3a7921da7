#!/bin/bash
# Mixed-step A/B of the residual+LN forms (NOMIC_RLN 222 vs 232), alternating, same box.
set -o pipefail
OUT=${OUT:-gpurun_out/rln_mixed}
mkdir -p "$OUT"
for r in 1 2 3; do
  for v in 222 232; do
    NOMIC_RLN=$v timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --host-api 0 --host-api-threads2 0 \
      --search-keys 0 --daemon-docs 0 --embed-e2e 0 > "$OUT/bench_${v}_$r.out" 2>/dev/null || exit 1
    python3 -c "import json; d=json.loads(open('$OUT/bench_${v}_$r.out').read().strip().splitlines()[-1]); print('$v', '$r', round(d['ms_per_step'], 3), round(d['value'] / 1e9, 4))"
  done
done
