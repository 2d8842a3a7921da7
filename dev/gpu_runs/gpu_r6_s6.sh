#!/bin/bash
# exchange phase attribution (2-rank peer vs 1-rank, one GPU), per-call floor (ring stamps build),
# qkv GEMM tile A/B (128^2 vs 256^2 on the 1152-tile shape) in the encoder
set -o pipefail
OUT=${OUT6:-gpurun_out/r6s6}
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
COMMON="--mode kv --steps 10 --warmup 3 --host-api 0 --host-api-threads2 0 --embed-e2e 0 --daemon-docs 0 --search-keys 0 --exchange-ab 0 --kv-async-ab 0 --mixed5 0 --verify 5000 --value-len 150"
SPLINTER_XR_PHASES=1 timeout -k 10 400 python -u bench.py --gpus 2 --keys-per-gpu 20000000 --batch 4000000 --backend gloo --transport peer $COMMON > $OUT/xr2.out 2> $OUT/xr2.err || { tail -30 $OUT/xr2.err; exit 1; }
python3 -c "import json; d=json.loads([l for l in open('$OUT/xr2.out') if l.startswith('{')][-1]); print('2rank', d['value']/1e9, d['ms_per_step'], d['integrity_failures']); print(json.dumps(d['xr_phases_ms']))"
timeout -k 10 400 python -u bench.py --gpus 1 --keys-per-gpu 40000000 --batch 8000000 $COMMON > $OUT/xr1.out 2> $OUT/xr1.err || { tail -30 $OUT/xr1.err; exit 1; }
python3 -c "import json; d=json.loads([l for l in open('$OUT/xr1.out') if l.startswith('{')][-1]); print('1rank', d['value']/1e9, d['ms_per_step'], d['integrity_failures'])"
for t in 1 16 32; do
  SPLINTER_HIP_VARIANT=stamps timeout -k 10 120 libsplinter_amd/bin/splinter_hostapi_bench --store hbm:stamp$t --threads $t --seconds 3 --keys 65536 --value-len 150 > $OUT/stamps_t$t.out 2> $OUT/stamps_t$t.err || { tail -5 $OUT/stamps_t$t.err; exit 1; }
  echo "t=$t"; cat $OUT/stamps_t$t.out; grep -E "stamps|seg_us|clock" $OUT/stamps_t$t.err
done
for t in 16 32; do
  timeout -k 10 120 libsplinter_amd/bin/splinter_hostapi_bench --store hbm:nost$t --threads $t --seconds 3 --keys 65536 --value-len 150 > $OUT/nostamps_t$t.out 2> $OUT/nostamps_t$t.err || exit 1
  echo "default t=$t"; cat $OUT/nostamps_t$t.out
done
EMB="--mode embed --steps 20 --warmup 5 --embed-e2e 0 --host-api 0 --host-api-threads2 0 --daemon-docs 0 --search-keys 0 --exchange-ab 0 --kv-async-ab 0 --mixed5 0"
for rep in 1 2; do
  for mt in 1024 2000; do
    NOMIC_GEMM256_MIN_TILES=$mt timeout -k 10 300 python -u bench.py $EMB > $OUT/emb_mt$mt.$rep.out 2> $OUT/emb_mt$mt.$rep.err || { tail -20 $OUT/emb_mt$mt.$rep.err; exit 1; }
    python3 -c "import json; d=json.loads([l for l in open('$OUT/emb_mt$mt.$rep.out') if l.startswith('{')][-1]); print('min_tiles=$mt rep=$rep', round(d['value'],1), 'vec/s', round(d['ms_per_step'],3), 'ms')"
  done
done
timeout -k 10 300 python -u -m pytest tests/test_nomic_gpu.py -k attention_varlen -q --timeout 120 --timeout-method thread > $OUT/attn_tests.txt 2>&1 || { tail -20 $OUT/attn_tests.txt; exit 1; }
tail -2 $OUT/attn_tests.txt
ATTN_VARIANTS=13,14,15,16 timeout -k 10 300 python -u scripts/attn_bench.py --rounds 7 > $OUT/attn_ab.jsonl 2> $OUT/attn_ab.err || { tail -10 $OUT/attn_ab.err; exit 1; }
cat $OUT/attn_ab.jsonl
