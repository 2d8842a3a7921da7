#!/bin/bash
# mixed step with the driver's arenas (25 M-key search arena as the encoder's document arena):
# serial phases vs the native KV fan-out overlapped with the encoder (unmasked), 3 alternating rounds
set -o pipefail
OUT=gpurun_out/r6s19
mkdir -p $OUT
B="--steps 30 --warmup 3 --embed-e2e 0 --host-api 0 --host-api-threads2 0 --daemon-docs 0 --exchange-ab 0 --kv-async-ab 0 --mixed5 0 --search-queries 0"
for rep in 1 2 3; do
  for c in serial ov0; do
    X=""; [ $c = ov0 ] && X="--overlap-native 1"
    timeout -k 10 500 python -u bench.py $B $X > $OUT/mix_$c.$rep.out 2> $OUT/mix_$c.$rep.err || { tail -20 $OUT/mix_$c.$rep.err; exit 1; }
    python3 -c "import json; d=json.loads([l for l in open('$OUT/mix_$c.$rep.out') if l.startswith('{')][-1]); print('$c rep=$rep', round(d['value']/1e9,4), 'G', round(d['ms_per_step'],3), 'ms enc', round(d.get('embed_phase_ms_per_step') or 0,3), 'integrity', d['integrity_failures'], d['timed_set_failures'])" | tee -a $OUT/summary.txt
  done
done
