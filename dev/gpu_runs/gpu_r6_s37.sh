#!/bin/bash
# GEMM tile-order band width (NOMIC_GEMM_GN: n-tiles per band of the XCD-remapped order) in the encoder
set -o pipefail
OUT=gpurun_out/r6s37
mkdir -p $OUT
EMB="--mode embed --steps 20 --warmup 5 --embed-e2e 0 --host-api 0 --host-api-threads2 0 --daemon-docs 0 --search-keys 0 --exchange-ab 0 --kv-async-ab 0 --mixed5 0"
for rep in 1 2 3; do
  for g in def 2 6 8 0; do
    E=""; [ $g != def ] && E="NOMIC_GEMM_GN=$g"
    env $E timeout -k 10 300 python -u bench.py $EMB > $OUT/emb_g$g.$rep.out 2> $OUT/emb_g$g.$rep.err || { tail -20 $OUT/emb_g$g.$rep.err; exit 1; }
    python3 -c "import json; d=json.loads([l for l in open('$OUT/emb_g$g.$rep.out') if l.startswith('{')][-1]); print('gn=$g rep=$rep', round(d['value'],1), 'vec/s', round(d['ms_per_step'],3), 'ms')" | tee -a $OUT/summary.txt
  done
done
