#!/bin/bash
# config #2's stream-posted server: wave-vote rounds inside a chunk (SPL_KVS_ASYNC_WV=1) vs the per-round
# workgroup barrier (0), against the fused grid; arena tests under the new server first
set -o pipefail
OUT=gpurun_out/r6s27
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_arena_gpu.py -x -q -k "kvs or async or server" --timeout 300 --timeout-method thread > $OUT/tests.txt 2>&1 || { tail -30 $OUT/tests.txt; exit 1; }
tail -1 $OUT/tests.txt
KV="--mode kv --steps 20 --warmup 5 --exchange-ab 0 --kv-async-ab 0 --host-api 0 --host-api-threads2 0"
for rep in 1 2 3; do
  for c in fused wv1 wv0 wv1_4096; do
    case $c in
      fused) E="SPL_KVS_FUSED=2";; wv1) E="SPL_KVS_FUSED=3 SPL_KVS_ASYNC_WV=1";; wv0) E="SPL_KVS_FUSED=3 SPL_KVS_ASYNC_WV=0";;
      wv1_4096) E="SPL_KVS_FUSED=3 SPL_KVS_ASYNC_WV=1 SPL_KVS_ASYNC_CHUNK=4096";;
    esac
    env $E timeout -k 10 300 python -u bench.py $KV > $OUT/kv_$c.$rep.out 2> $OUT/kv_$c.$rep.err || { tail -20 $OUT/kv_$c.$rep.err; exit 1; }
    python3 -c "import json; d=json.loads([l for l in open('$OUT/kv_$c.$rep.out') if l.startswith('{')][-1]); print('kv $c rep=$rep', round(d['value']/1e9,4), 'G', round(d['ms_per_step'],3), 'ms integrity', d['integrity_failures'], d['timed_set_failures'], 'again', d['kv_eagain_retries'], 'err', d.get('kv_async_error'))" | tee -a $OUT/summary.txt
  done
done
