#!/bin/bash
# One gpurun call, several checks (the pool is busy; calls are scarce): targeted GPU tests, fused
# KV modes 2 vs 3, encoder interference (shared server vs CPU-only clients), timed-region traces
# of the native and routed step, KV PMC split.  Stops at the first failing step.
set -o pipefail
OUT=${OUT:-gpurun_out/r4k}
mkdir -p "$OUT"
step() {
  local name=$1; shift
  "$@" > "$OUT/$name.out" 2> "$OUT/$name.err"
  local rc=$?
  echo "== $name rc=$rc"; tail -c 1200 "$OUT/$name.out"
  if [ $rc -ne 0 ]; then tail -20 "$OUT/$name.err"; exit $rc; fi
}
step pre_tests timeout -k 10 600 python -u -m pytest tests/test_batch_api.py tests/test_ring_gpu.py tests/test_arena_gpu.py \
  -x -v -m gpu --timeout 150 --timeout-method thread
step attn_tests timeout -k 10 300 python -u -m pytest tests/test_nomic_gpu.py -x -v -k attention --timeout 150 \
  --timeout-method thread
step attn_bench env ATTN_VARIANTS=13,14 timeout -k 10 200 python -u scripts/attn_bench.py --rounds 7
for f in 2 3; do
  step kv_fused$f env SPL_KVS_FUSED=$f timeout -k 10 300 python -u bench.py --mode kv --steps 20 --warmup 5 \
    --host-api 0 --host-api-threads2 0 --routed-steps 0
done
step interf timeout -k 10 400 python -u scripts/ring_interference.py --clients 4 --threads 1,2 --modes shared,cpu --steps 20
OUT=$OUT/trace ./scripts/gpu_trace_routed.sh > "$OUT/trace.log" 2>&1 || { tail -30 "$OUT/trace.log"; exit 1; }
tail -60 "$OUT/trace.log"
OUT=$OUT/pmc ./scripts/gpu_pmc_kv.sh > "$OUT/pmc.log" 2>&1 || { tail -30 "$OUT/pmc.log"; exit 1; }
tail -30 "$OUT/pmc.log"
exit 0
