# round 2, call 24: post-KV embed slowdown vs the number of hardware queues in use
set -x
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r2_24
mkdir -p $O
B="--writer-streams 1 --reader-streams 1 --mop 1 --host-api 0"
F="SPLINTER_HBM_NO_RING=1 BENCH_SKIP_MOP=1 BENCH_PY_STREAMS=1"
run() { tag=$1; shift; env "$@" timeout -k 10 200 python bench.py $B > $O/$tag.json 2> $O/$tag.err; }
run fast SPLINTER_HBM_NO_RING=1 BENCH_SKIP_MOP=1 BENCH_PY_STREAMS=1 &&
run fast_x2high SPLINTER_HBM_NO_RING=1 BENCH_SKIP_MOP=1 BENCH_PY_STREAMS=1 BENCH_EXTRA_STREAMS=2 &&
run fast_x2normal SPLINTER_HBM_NO_RING=1 BENCH_SKIP_MOP=1 BENCH_PY_STREAMS=1 BENCH_EXTRA_STREAMS=2 BENCH_EXTRA_PRIO=normal &&
run default_q2 GPU_MAX_HW_QUEUES=2 &&
run default_q1 GPU_MAX_HW_QUEUES=1 &&
run default X=1 &&
echo done
