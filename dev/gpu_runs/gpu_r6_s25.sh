#!/bin/bash
# fused KV grid: fixed lane streams + wave-vote exit with the last 1/16 .. 4/16 of the batch claimed by
# waves in 128 / 256 / 512-row chunks (4), vs workgroup chunks (1, default) and fixed streams with the
# wave-vote exit (3); tests under form 4 first, then the mixed step for the best forms
set -o pipefail
OUT=gpurun_out/r6s25
mkdir -p $OUT
SPL_KVS_DYN=4 timeout -k 10 600 python -u -m pytest tests/test_arena_gpu.py tests/test_route_gpu.py -x -q --timeout 300 --timeout-method thread > $OUT/tests.txt 2>&1 || { tail -30 $OUT/tests.txt; exit 1; }
tail -1 $OUT/tests.txt
KV="--mode kv --steps 20 --warmup 5 --exchange-ab 0 --kv-async-ab 0 --host-api 0 --host-api-threads2 0"
for rep in 1 2 3; do
  for c in d1 d3 d4_2_256 d4_1_256 d4_4_256 d4_2_128 d4_2_512; do
    case $c in
      d1) E="SPL_KVS_DYN=1";; d3) E="SPL_KVS_DYN=3";;
      d4_*) x=${c#d4_}; E="SPL_KVS_DYN=4 SPL_KVS_DYN_TAIL16=${x%_*} SPL_KVS_DYN_TCHUNK=${x#*_}";;
    esac
    env $E timeout -k 10 300 python -u bench.py $KV > $OUT/kv_$c.$rep.out 2> $OUT/kv_$c.$rep.err || { tail -20 $OUT/kv_$c.$rep.err; exit 1; }
    python3 -c "import json; d=json.loads([l for l in open('$OUT/kv_$c.$rep.out') if l.startswith('{')][-1]); print('kv $c rep=$rep', round(d['value']/1e9,4), 'G', round(d['ms_per_step'],3), 'ms integrity', d['integrity_failures'], d['timed_set_failures'], 'again', d['kv_eagain_retries'])" | tee -a $OUT/summary.txt
  done
done
