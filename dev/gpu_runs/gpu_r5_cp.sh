#!/bin/bash
# command-processor-woken worker probe (scripts/probes/cpwait_probe.hip), twice
set -o pipefail
OUT=gpurun_out/r5cp
mkdir -p $OUT
hipcc --offload-arch=gfx950 -O2 -o $OUT/cpwait_probe scripts/probes/cpwait_probe.hip 2> $OUT/build.err || { tail -5 $OUT/build.err; exit 1; }
for r in 1 2; do
  timeout -k 10 120 $OUT/cpwait_probe > $OUT/cpwait.$r.jsonl 2> $OUT/cpwait.$r.err || { cat $OUT/cpwait.$r.jsonl; tail -5 $OUT/cpwait.$r.err; exit 1; }
  cat $OUT/cpwait.$r.jsonl
done
