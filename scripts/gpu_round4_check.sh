#!/bin/bash
# Round-4 GPU validation on one MI355X (run through gpurun from the repo root): the GPU test
# suite, the 1-GPU headline bench, a 2-rank routed-exchange rehearsal (both ranks on device 0,
# peer transport, gloo for the small collectives) and a profile of the host-array batch ABI.
# Every GPU step has its own time limit; the script stops at the first step that fails.
set -o pipefail
OUT=${OUT:-gpurun_out/r4}
mkdir -p "$OUT"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || { echo "pytest failed rc=$?"; tail -30 "$OUT/pytest_gpu.log"; exit 1; }
tail -3 "$OUT/pytest_gpu.log"
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > "$OUT/bench.json" 2> "$OUT/bench.err" || { echo "bench failed"; tail -20 "$OUT/bench.err"; exit 1; }
cat "$OUT/bench.json"
timeout -k 10 300 python -u bench.py --gpus 2 --backend gloo --mode kv --keys-per-gpu 20000000 --batch 4000000 \
  --steps 10 --warmup 3 --search-keys 0 --host-api 0 --host-api-threads2 0 --routed-steps 0 \
  > "$OUT/bench2.json" 2> "$OUT/bench2.err" || { echo "bench2 failed"; tail -20 "$OUT/bench2.err"; exit 1; }
cat "$OUT/bench2.json"
