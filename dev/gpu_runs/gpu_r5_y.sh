#!/bin/bash
# round-5 validation: full GPU suite, smoke, the default bench (driver arguments)
set -o pipefail
OUT=gpurun_out/r5y
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.txt 2>&1 || { tail -30 $OUT/pytest_gpu.txt; exit 1; }
tail -3 $OUT/pytest_gpu.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.txt 2>&1 || { tail -20 $OUT/smoke.txt; exit 1; }
tail -1 $OUT/smoke.txt
timeout -k 10 900 python bench.py > $OUT/bench.out 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
tail -1 $OUT/bench.out
# command-processor-woken worker probe (scripts/probes/cpwait_probe.hip)
hipcc --offload-arch=gfx950 -O2 -o $OUT/cpwait_probe scripts/probes/cpwait_probe.hip 2> $OUT/cpwait_build.err || { tail -5 $OUT/cpwait_build.err; exit 1; }
timeout -k 10 120 $OUT/cpwait_probe > $OUT/cpwait.jsonl 2> $OUT/cpwait.err || { tail -5 $OUT/cpwait.err; exit 1; }
cat $OUT/cpwait.jsonl
