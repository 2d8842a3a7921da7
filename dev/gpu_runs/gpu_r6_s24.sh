#!/bin/bash
# fused KV grid: workgroup chunks (1, default) vs per-wave chunks with a wave-vote loop exit (2, chunk
# 512 / 1024 / 2048 rows per wave claim) vs fixed lane streams with the wave-vote exit (3) vs fixed
# lane streams with the workgroup barrier (0); tests under form 2 first
set -o pipefail
OUT=gpurun_out/r6s24
mkdir -p $OUT
SPL_KVS_DYN=2 timeout -k 10 600 python -u -m pytest tests/test_arena_gpu.py tests/test_route_gpu.py -x -q --timeout 300 --timeout-method thread > $OUT/tests.txt 2>&1 || { tail -30 $OUT/tests.txt; exit 1; }
tail -1 $OUT/tests.txt
KV="--mode kv --steps 20 --warmup 5 --exchange-ab 0 --kv-async-ab 0 --host-api 0 --host-api-threads2 0"
for rep in 1 2 3; do
  for c in d1 d2_1024 d2_512 d2_2048 d3 d0; do
    case $c in
      d1) E="SPL_KVS_DYN=1";; d3) E="SPL_KVS_DYN=3";; d0) E="SPL_KVS_DYN=0";;
      d2_*) E="SPL_KVS_DYN=2 SPL_KVS_DYN_WCHUNK=${c#d2_}";;
    esac
    env $E timeout -k 10 300 python -u bench.py $KV > $OUT/kv_$c.$rep.out 2> $OUT/kv_$c.$rep.err || { tail -20 $OUT/kv_$c.$rep.err; exit 1; }
    python3 -c "import json; d=json.loads([l for l in open('$OUT/kv_$c.$rep.out') if l.startswith('{')][-1]); print('kv $c rep=$rep', round(d['value']/1e9,4), 'G', round(d['ms_per_step'],3), 'ms integrity', d['integrity_failures'], d['timed_set_failures'], 'again', d['kv_eagain_retries'])" | tee -a $OUT/summary.txt
  done
done
