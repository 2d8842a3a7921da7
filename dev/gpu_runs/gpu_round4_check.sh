#!/bin/bash
# Round-4 GPU validation on one MI355X (run through gpurun from the repo root): the 1-GPU headline
# bench, a 2-rank routed-exchange rehearsal (both ranks on device 0, peer transport, gloo for the
# small collectives), the host-array batch ABI, optional A/B experiments, then the GPU test suite.
# Every GPU step has its own time limit; a timeout, crash or abort ends the script (test failures,
# pytest rc 1, do not).
set -o pipefail
OUT=${OUT:-gpurun_out/r4}
mkdir -p "$OUT"
step() {  # step NAME CMD... : run with output to $OUT/NAME.{out,err}; stop on rc != 0
  local name=$1; shift
  "$@" > "$OUT/$name.out" 2> "$OUT/$name.err"
  local rc=$?
  echo "== $name rc=$rc"; tail -c 3000 "$OUT/$name.out"
  if [ $rc -ne 0 ]; then tail -20 "$OUT/$name.err"; exit $rc; fi
}
if [ -n "$PRE_TESTS" ]; then  # targeted tests first (new code), fail fast
  step pre_tests timeout -k 10 600 python -u -m pytest $PRE_TESTS -x -v --timeout 150 --timeout-method thread
fi
if [ -n "$EXTRA_RING" ]; then
  # per-call API: one process at 1 / 32 / 64 threads, 4 processes x 8 / 16 threads on the owner's ring
  # server (default) and with a worker per process (SPLINTER_RING_SHARED=0); encoder beside 4 clients
  H=./libsplinter_amd/bin/splinter_hostapi_bench
  for t in 1 32 64; do step ring_t$t timeout -k 10 120 $H --store hbm:rt$t --threads $t --seconds 2 --keys 20000; done
  for t in 32 64; do
    step ring_t${t}_private env SPLINTER_RING_SHARED=0 timeout -k 10 120 $H --store hbm:ru$t --threads $t --seconds 2 \
      --keys 20000
  done
  for t in 8 16; do
    step ring_p4t${t}_shared timeout -k 10 120 $H --store hbm:rp$t --procs 4 --threads $t --seconds 2 --keys 20000
    step ring_p4t${t}_private env SPLINTER_RING_SHARED=0 timeout -k 10 120 $H --store hbm:rq$t --procs 4 --threads $t \
      --seconds 2 --keys 20000
  done
  step ring_interference timeout -k 10 300 python -u scripts/ring_interference.py --clients 4 --threads ${RI_THREADS:-1,2,8} \
    --steps 20
fi
if [ -z "$SKIP_BENCH" ]; then
  step bench timeout -k 10 300 python -u bench.py --steps 20 --warmup 5
  step bench2 timeout -k 10 300 python -u bench.py --gpus 2 --backend gloo --mode kv --keys-per-gpu 20000000 \
    --batch 4000000 --steps 10 --warmup 3 --search-keys 0 --host-api 0 --host-api-threads2 0 --routed-steps 0
fi
if [ -n "$EXTRA_BATCH" ]; then
  for st in hbm:xb1 node:xb2; do
    step batch_${st%%:*} env SPLINTER_NODE_SHARDS=4 timeout -k 10 120 ./libsplinter_amd/bin/splinter_hostapi_bench \
      --store $st --batch 2000000 --keys 8000000 --seconds 3
  done
fi
if [ -n "$EXTRA_PROF" ]; then
  # kernel + memory-copy trace of the batch ABI on hbm: (where the host-array batch time goes)
  (cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT" && timeout -k 10 120 rocprofv3 --kernel-trace --memory-copy-trace \
    --stats -d "$OUT/prof_batch" -o run -- ./libsplinter_amd/bin/splinter_hostapi_bench --store hbm:xb3 --batch 2000000 \
    --keys 4000000 --seconds 2 > "$OUT/batch_prof.out" 2>&1) || { echo "batch profile failed"; exit 1; }
fi
if [ -n "$EXTRA_KV" ]; then
  for f in ${KV_MODES:-0 1 2}; do
    step bench_kv_fused$f env SPL_KVS_FUSED=$f timeout -k 10 300 python -u bench.py --mode kv --steps 20 --warmup 5 \
      --host-api 0 --host-api-threads2 0 --routed-steps 0
  done
fi
if [ -n "$EXTRA_OVERLAP" ]; then
  step bench_overlap timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --overlap-native 1 --embed-e2e 0 \
    --host-api 0 --host-api-threads2 0 --daemon-docs 0 --routed-steps 0
fi
if [ -n "$SMOKE" ]; then
  step smoke timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()"
fi
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 150 --timeout-method thread ${PYTEST_ARGS} \
    > "$OUT/pytest_gpu.log" 2>&1
  rc=$?; tail -15 "$OUT/pytest_gpu.log"; echo "pytest rc=$rc"
fi
exit 0
