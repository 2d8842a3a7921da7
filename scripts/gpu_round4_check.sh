#!/bin/bash
# Round-4 GPU validation on one MI355X (run through gpurun from the repo root): the GPU test
# suite, the 1-GPU headline bench, a 2-rank routed-exchange rehearsal (both ranks on device 0,
# peer transport, gloo for the small collectives) and the host-array batch ABI.
# Every GPU step has its own time limit.  Test failures (pytest rc 1) do not stop the later steps;
# a timeout, crash or abort does.
set -o pipefail
OUT=${OUT:-gpurun_out/r4}
mkdir -p "$OUT"
fatal() { case "$1" in 0|1) return 1;; *) return 0;; esac; }
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread ${PYTEST_ARGS} > "$OUT/pytest_gpu.log" 2>&1
rc=$?; tail -15 "$OUT/pytest_gpu.log"; if fatal $rc; then echo "pytest rc=$rc: stopping"; exit $rc; fi
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > "$OUT/bench.json" 2> "$OUT/bench.err"
rc=$?; cat "$OUT/bench.json"; if [ $rc -ne 0 ]; then tail -20 "$OUT/bench.err"; exit $rc; fi
timeout -k 10 300 python -u bench.py --gpus 2 --backend gloo --mode kv --keys-per-gpu 20000000 --batch 4000000 \
  --steps 10 --warmup 3 --search-keys 0 --host-api 0 --host-api-threads2 0 --routed-steps 0 \
  > "$OUT/bench2.json" 2> "$OUT/bench2.err"
rc=$?; cat "$OUT/bench2.json"; if [ $rc -ne 0 ]; then tail -20 "$OUT/bench2.err"; exit $rc; fi
for st in hbm:xb1 node:xb2; do
  SPLINTER_NODE_SHARDS=4 timeout -k 10 120 ./libsplinter_amd/bin/splinter_hostapi_bench --store $st --batch 2000000 \
    --keys 8000000 --seconds 3 >> "$OUT/batch_api.jsonl" 2>&1 || { echo "batch $st failed"; exit 1; }
done
cat "$OUT/batch_api.jsonl"
if [ -n "$EXTRA_PROF" ]; then
  # kernel + memory-copy trace of the batch ABI on hbm: (where the host-array batch time goes)
  (cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT" && timeout -k 10 120 rocprofv3 --kernel-trace --memory-copy-trace \
    --stats -d "$OUT/prof_batch" -o run -- ./libsplinter_amd/bin/splinter_hostapi_bench --store hbm:xb3 --batch 2000000 \
    --keys 4000000 --seconds 2 > "$OUT/batch_prof.json" 2>&1) || { echo "batch profile failed"; exit 1; }
fi
if [ -n "$EXTRA_OVERLAP" ]; then
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --overlap-native 1 --embed-e2e 0 --host-api 0 \
    --host-api-threads2 0 --daemon-docs 0 --routed-steps 0 > "$OUT/bench_overlap.json" 2> "$OUT/bench_overlap.err"
  rc=$?; cat "$OUT/bench_overlap.json"; [ $rc -ne 0 ] && { tail -20 "$OUT/bench_overlap.err"; exit $rc; }
fi
if [ -n "$EXTRA_KV" ]; then
  for f in 0 1 2; do
    SPL_KVS_FUSED=$f timeout -k 10 300 python -u bench.py --mode kv --steps 20 --warmup 5 --host-api 0 \
      --host-api-threads2 0 --routed-steps 0 > "$OUT/bench_kv_fused$f.json" 2> "$OUT/bench_kv_fused$f.err"
    rc=$?; cat "$OUT/bench_kv_fused$f.json"; [ $rc -ne 0 ] && { tail -20 "$OUT/bench_kv_fused$f.err"; exit $rc; }
  done
fi
exit 0
