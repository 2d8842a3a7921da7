#!/bin/bash
# k_attn3 at 4 waves per SIMD (<= 128 VGPRs, 13 spilled; NOMIC_ATTN=20) vs 3 (152 VGPRs, default 13)
set -o pipefail
OUT=gpurun_out/r6s30
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_nomic_gpu.py -k attention_varlen -q --timeout 120 --timeout-method thread > $OUT/attn_tests.txt 2>&1 || { tail -30 $OUT/attn_tests.txt; exit 1; }
tail -1 $OUT/attn_tests.txt
ATTN_VARIANTS=13,20 timeout -k 10 300 python -u scripts/attn_bench.py --rounds 9 > $OUT/attn_bench.jsonl 2> $OUT/attn_bench.err || { tail -20 $OUT/attn_bench.err; exit 1; }
cat $OUT/attn_bench.jsonl
EMB="--mode embed --steps 20 --warmup 5 --embed-e2e 0 --host-api 0 --host-api-threads2 0 --daemon-docs 0 --search-keys 0 --exchange-ab 0 --kv-async-ab 0 --mixed5 0"
for rep in 1 2 3; do
  for v in 13 20; do
    NOMIC_ATTN=$v timeout -k 10 300 python -u bench.py $EMB > $OUT/emb_a$v.$rep.out 2> $OUT/emb_a$v.$rep.err || { tail -20 $OUT/emb_a$v.$rep.err; exit 1; }
    python3 -c "import json; d=json.loads([l for l in open('$OUT/emb_a$v.$rep.out') if l.startswith('{')][-1]); print('attn=$v rep=$rep', round(d['value'],1), 'vec/s', round(d['ms_per_step'],3), 'ms')" | tee -a $OUT/summary.txt
  done
done
