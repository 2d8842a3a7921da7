#!/bin/bash
# direct routed responses: route tests (both modes), then the exchange A/B (2 ranks on one GPU vs 1 rank)
set -o pipefail
OUT=gpurun_out/r6s12
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/test_route_gpu.py -v --timeout 300 --timeout-method thread > $OUT/route.txt 2>&1
rc=$?; grep -E "PASSED|FAILED|^E " $OUT/route.txt | cut -c1-300 | tail -20
[ $rc -eq 0 ] || exit 1
COMMON="--mode kv --steps 10 --warmup 3 --host-api 0 --host-api-threads2 0 --embed-e2e 0 --daemon-docs 0 --search-keys 0 --exchange-ab 0 --kv-async-ab 0 --mixed5 0 --verify 5000 --value-len 150"
for rep in 1 2; do
  for d in 1 0; do
    SPLINTER_XR_DIRECT=$d SPLINTER_XR_PHASES=1 timeout -k 10 400 python -u bench.py --gpus 2 --keys-per-gpu 20000000 --batch 4000000 --backend gloo --transport peer $COMMON > $OUT/xr2_d$d.$rep.out 2> $OUT/xr2_d$d.$rep.err || { tail -30 $OUT/xr2_d$d.$rep.err; exit 1; }
    python3 -c "import json; d=json.loads([l for l in open('$OUT/xr2_d$d.$rep.out') if l.startswith('{')][-1]); print('direct=$d rep=$rep', round(d['value']/1e9,4), 'G', round(d['ms_per_step'],3), 'ms integrity', d['integrity_failures'], json.dumps(d['xr_phases_ms']))"
  done
done
timeout -k 10 400 python -u bench.py --gpus 1 --keys-per-gpu 40000000 --batch 8000000 $COMMON > $OUT/xr1.out 2> $OUT/xr1.err || { tail -30 $OUT/xr1.err; exit 1; }
python3 -c "import json; d=json.loads([l for l in open('$OUT/xr1.out') if l.startswith('{')][-1]); print('1rank', round(d['value']/1e9,4), 'G', round(d['ms_per_step'],3), 'ms integrity', d['integrity_failures'])"
