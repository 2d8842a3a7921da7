#!/bin/bash
# mixed step with the driver's arenas: fused KV grid forms 0 (fixed streams, workgroup barrier), 1
# (workgroup chunks), 3 (fixed streams, wave-vote exit), 4 (3 + the last 2/16 claimed in 512-row wave
# chunks), 3 alternating rounds
set -o pipefail
OUT=gpurun_out/r6s26
mkdir -p $OUT
B="--steps 30 --warmup 3 --embed-e2e 0 --host-api 0 --host-api-threads2 0 --daemon-docs 0 --exchange-ab 0 --kv-async-ab 0 --mixed5 0 --search-queries 0"
for rep in 1 2 3; do
  for c in 0 1 3 4; do
    E="SPL_KVS_DYN=$c"; [ $c = 4 ] && E="SPL_KVS_DYN=4 SPL_KVS_DYN_TAIL16=2 SPL_KVS_DYN_TCHUNK=512"
    env $E timeout -k 10 500 python -u bench.py $B > $OUT/mix_$c.$rep.out 2> $OUT/mix_$c.$rep.err || { tail -20 $OUT/mix_$c.$rep.err; exit 1; }
    python3 -c "import json; d=json.loads([l for l in open('$OUT/mix_$c.$rep.out') if l.startswith('{')][-1]); print('mixed d$c rep=$rep', round(d['value']/1e9,4), 'G', round(d['ms_per_step'],3), 'ms integrity', d['integrity_failures'], d['timed_set_failures'], 'again', d['kv_eagain_retries'])" | tee -a $OUT/summary.txt
  done
done
