#!/bin/bash
# round-6 validation: GPU suite, smoke, default bench, timed-region kernel trace of the mixed step
set -o pipefail
OUT=${OUTF:-gpurun_out/r6final}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 1200 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.txt 2>&1; echo "suite rc=$?"
tail -4 $OUT/pytest_gpu.txt
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.txt 2>&1 || { tail -20 $OUT/smoke.txt; exit 1; }
tail -1 $OUT/smoke.txt
timeout -k 10 900 python -u bench.py > $OUT/bench.out 2> $OUT/bench.err || { tail -30 $OUT/bench.err; exit 1; }
tail -c 1500 $OUT/bench.out
ARGS="--steps 10 --warmup 3 --embed-e2e 0 --host-api 0 --host-api-threads2 0 --daemon-docs 0 --exchange-ab 0 --kv-async-ab 0 --mixed5 0"
SPL_PROFILE_TIMED=1 timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $PWD/$OUT/tr_native -o run -- python3 bench.py $ARGS > $OUT/trace.out 2> $OUT/trace.err || { tail -20 $OUT/trace.err; exit 1; }
csv=$(find $OUT/tr_native -name '*kernel_trace.csv' | head -1)
python3 scripts/trace_window.py "$csv" $OUT/trace.err --md $OUT/trace_native.md --timeline || exit 1
rm -f "$csv"
head -20 $OUT/trace_native.md
