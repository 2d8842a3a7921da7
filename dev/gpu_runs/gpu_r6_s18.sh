#!/bin/bash
# mixed step: serial phases vs the native KV fan-out overlapped with the encoder, KV grid unmasked or
# confined to 8 / 16 / 24 CUs per XCD (encoder on every CU); arena tests first (CU-aware grid sizing)
set -o pipefail
OUT=gpurun_out/r6s18
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_arena_gpu.py -x -q --timeout 300 --timeout-method thread > $OUT/tests.txt 2>&1 || { tail -20 $OUT/tests.txt; exit 1; }
tail -1 $OUT/tests.txt
B="--steps 20 --warmup 5 --embed-e2e 0 --host-api 0 --host-api-threads2 0 --daemon-docs 0 --search-keys 0 --exchange-ab 0 --kv-async-ab 0 --mixed5 0"
for rep in 1 2; do
  for c in serial ov0 ov16 ov8 ov24; do
    case $c in
      serial) X="";;
      ov0) X="--overlap-native 1";;
      ov*) X="--overlap-native 1 --overlap-kv-cus ${c#ov}";;
    esac
    timeout -k 10 400 python -u bench.py $B $X > $OUT/mix_$c.$rep.out 2> $OUT/mix_$c.$rep.err || { tail -20 $OUT/mix_$c.$rep.err; exit 1; }
    python3 -c "import json; d=json.loads([l for l in open('$OUT/mix_$c.$rep.out') if l.startswith('{')][-1]); print('$c rep=$rep', round(d['value']/1e9,4), 'G', round(d['ms_per_step'],3), 'ms enc', round(d.get('embed_phase_ms_per_step') or 0,3), 'integrity', d['integrity_failures'], d['timed_set_failures'], 'again', d['kv_eagain_retries'])" | tee -a $OUT/summary.txt
  done
done
