#!/bin/bash
# Ring at its round-4 defaults (normal-priority worker queue, hold API): ring GPU tests, per-call
# latency / throughput, encoder beside live clients with and without a ring hold per step.
set -o pipefail
OUT=${OUT:-gpurun_out/r4z}
mkdir -p "$OUT"
step() {
  local name=$1; shift
  "$@" > "$OUT/$name.out" 2> "$OUT/$name.err"
  local rc=$?
  echo "== $name rc=$rc"; tail -c 700 "$OUT/$name.out"
  if [ $rc -ne 0 ]; then tail -20 "$OUT/$name.err"; exit $rc; fi
}
step ring_tests timeout -k 10 400 python -u -m pytest tests/test_ring_gpu.py -x -v --timeout 150 --timeout-method thread
H=./libsplinter_amd/bin/splinter_hostapi_bench
for t in 1 16 32 64; do step ring_t$t timeout -k 10 120 $H --store hbm:rz$t --threads $t --seconds 2 --keys 20000; done
step ring_p4t8 timeout -k 10 120 $H --store hbm:rzp --procs 4 --threads 8 --seconds 2 --keys 20000
step interf timeout -k 10 400 python -u scripts/ring_interference.py --clients 4 --threads 1,2 --steps 20 \
  --modes shared,held --settle 2
exit 0
