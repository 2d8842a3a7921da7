#!/bin/bash
# maintenance window tests; per-call floor with the ring stamps backend (SPLINTER_HIP_LIB); attention
# form 16 vs 13 inside the encoder
set -o pipefail
OUT=gpurun_out/r6s9
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_maint_gpu.py -k "online_beside or open_maintenance_window" -v -s --timeout 300 --timeout-method thread > $OUT/maint.txt 2>&1
rc=$?; grep -E "PASSED|FAILED|^E " $OUT/maint.txt | cut -c1-300 | tail -12; grep -o "overlapped_steps[^r]*" $OUT/maint.txt; grep -o "dead_status[^l]*" $OUT/maint.txt
[ $rc -le 1 ] || exit 1
STAMPS=$PWD/libsplinter_amd/lib/libsplinter_hip_stamps.so
for t in 1 16 32; do
  SPLINTER_HIP_LIB=$STAMPS timeout -k 10 120 libsplinter_amd/bin/splinter_hostapi_bench --store hbm:stamp$t --threads $t --seconds 3 --keys 65536 --value-len 150 > $OUT/stamps_t$t.out 2> $OUT/stamps_t$t.err || { tail -5 $OUT/stamps_t$t.err; exit 1; }
  echo "t=$t"; cat $OUT/stamps_t$t.out; cat $OUT/stamps_t$t.err | head -8
done
EMB="--mode embed --steps 20 --warmup 5 --embed-e2e 0 --host-api 0 --host-api-threads2 0 --daemon-docs 0 --search-keys 0 --exchange-ab 0 --kv-async-ab 0 --mixed5 0"
for rep in 1 2 3; do
  for v in 13 16; do
    NOMIC_ATTN=$v timeout -k 10 300 python -u bench.py $EMB > $OUT/emb_a$v.$rep.out 2> $OUT/emb_a$v.$rep.err || { tail -20 $OUT/emb_a$v.$rep.err; exit 1; }
    python3 -c "import json; d=json.loads([l for l in open('$OUT/emb_a$v.$rep.out') if l.startswith('{')][-1]); print('attn=$v rep=$rep', round(d['value'],1), 'vec/s', round(d['ms_per_step'],3), 'ms')"
  done
done
