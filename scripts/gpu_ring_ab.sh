#!/bin/bash
# Ring-server A/B on one MI355X: worker waves (SPLINTER_RING_GROUPS), each with the per-call
# throughput bench at 1 / 32 / 64 threads and 4 processes, and the encoder-beside-clients
# interference run; then the node batch with its phase trace.  Stops at the first failing step.
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
for g in ${GROUPS_LIST:-4 8 32}; do
  for t in 1 32 64; do
    step t${t}_g$g env SPLINTER_RING_GROUPS=$g timeout -k 10 120 $H --store hbm:ab$t --threads $t --seconds 2 --keys 20000
  done
  step p4t8_g$g env SPLINTER_RING_GROUPS=$g timeout -k 10 120 $H --store hbm:ac --procs 4 --threads 8 --seconds 2 \
    --keys 20000
  step interf_g$g env SPLINTER_RING_GROUPS=$g timeout -k 10 300 python -u scripts/ring_interference.py --clients 4 \
    --threads 1,2 --steps 20
done
step batch_node_trace env SPLINTER_NODE_SHARDS=4 SPLINTER_NODE_BATCH_TRACE=1 timeout -k 10 120 $H --store node:xt \
  --batch 2000000 --keys 8000000 --seconds 3
exit 0
