#!/bin/bash
# Ring-server A/B on one MI355X: hipHostRegister flags of the shared segment and a CU-masked
# worker queue (SPLINTER_RING_REG_FLAGS / SPLINTER_RING_CUS), each with the per-call throughput
# bench and the encoder-beside-clients interference run.  Stops at the first failing step.
set -o pipefail
OUT=${OUT:-gpurun_out/ring_ab}
mkdir -p "$OUT"
H=./libsplinter_amd/bin/splinter_hostapi_bench
step() {
  local name=$1; shift
  "$@" > "$OUT/$name.out" 2> "$OUT/$name.err"
  local rc=$?
  echo "== $name rc=$rc"; tail -c 1500 "$OUT/$name.out"
  if [ $rc -ne 0 ]; then tail -20 "$OUT/$name.err"; exit $rc; fi
}
for rf in 2 0x80000002; do
  for t in 32 64; do
    step t${t}_rf$rf env SPLINTER_RING_REG_FLAGS=$rf timeout -k 10 120 $H --store hbm:ab$t --threads $t --seconds 2 --keys 20000
  done
  step p4t8_rf$rf env SPLINTER_RING_REG_FLAGS=$rf timeout -k 10 120 $H --store hbm:ac --procs 4 --threads 8 --seconds 2 \
    --keys 20000
done
step t32_private env SPLINTER_RING_SHARED=0 timeout -k 10 120 $H --store hbm:ad --threads 32 --seconds 2 --keys 20000
for cus in 0 8 32; do
  step t32_cus$cus env SPLINTER_RING_CUS=$cus timeout -k 10 120 $H --store hbm:ae$cus --threads 32 --seconds 2 --keys 20000
  step interf_cus$cus env SPLINTER_RING_CUS=$cus timeout -k 10 300 python -u scripts/ring_interference.py --clients 4 \
    --threads 1,2 --steps 20
done
exit 0
