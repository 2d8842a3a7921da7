#!/bin/bash
# Where the encoder's slowdown beside per-call clients comes from (gets only / sets only / a resident
# idle worker), and the 256-tile GEMM threshold A/B on embed-only steps.  One MI355X.
set -o pipefail
OUT=${OUT:-gpurun_out/r4l}
mkdir -p "$OUT"
step() {
  local name=$1; shift
  "$@" > "$OUT/$name.out" 2> "$OUT/$name.err"
  local rc=$?
  echo "== $name rc=$rc"; tail -c 900 "$OUT/$name.out"
  if [ $rc -ne 0 ]; then tail -20 "$OUT/$name.err"; exit $rc; fi
}
RI="python -u scripts/ring_interference.py --clients 4 --threads 1 --steps 20"
step interf_get timeout -k 10 300 $RI --modes shared --client-args "--set-frac 0"
step interf_set timeout -k 10 300 $RI --modes shared --client-args "--set-frac 1"
step interf_idle env SPLINTER_RING_IDLE_US=60000000 timeout -k 10 300 $RI --modes idle,shared
for r in 1 2; do
  for t in 1024 2048; do
    step embed_t${t}_$r env NOMIC_GEMM256_MIN_TILES=$t timeout -k 10 300 python -u bench.py --mode embed --steps 20 \
      --warmup 5
  done
done
exit 0
