#!/bin/bash
# direct responses: step ordering by device-side posts (flags) vs gloo-staged collectives
set -o pipefail
OUT=gpurun_out/r6s13
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
COMMON="--mode kv --steps 10 --warmup 3 --host-api 0 --host-api-threads2 0 --embed-e2e 0 --daemon-docs 0 --search-keys 0 --exchange-ab 0 --kv-async-ab 0 --mixed5 0 --verify 5000 --value-len 150"
for rep in 1 2; do
  for sy in flags coll; do
    SPLINTER_XR_SYNC=$sy SPLINTER_XR_PHASES=1 timeout -k 10 400 python -u bench.py --gpus 2 --keys-per-gpu 20000000 --batch 4000000 --backend gloo --transport peer $COMMON > $OUT/xr2_$sy.$rep.out 2> $OUT/xr2_$sy.$rep.err || { tail -30 $OUT/xr2_$sy.$rep.err; exit 1; }
    python3 -c "import json; d=json.loads([l for l in open('$OUT/xr2_$sy.$rep.out') if l.startswith('{')][-1]); print('sync=$sy rep=$rep', round(d['value']/1e9,4), 'G', round(d['ms_per_step'],3), 'ms integrity', d['integrity_failures'], 'err', d.get('xr_sync_error'), json.dumps(d['xr_phases_ms']))"
  done
done
