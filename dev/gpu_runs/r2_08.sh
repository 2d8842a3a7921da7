# round 2, call 8: why the embed phase is slower after the KV phase (mop, stream count, idle gap)
set -x
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r2_08
mkdir -p $O
run() { tag=$1; shift; timeout -k 10 200 python bench.py --host-api 0 "$@" > $O/$tag.json 2> $O/$tag.err; }
run ws1_mop0 --writer-streams 1 --reader-streams 1 --mop 0 &&
run ws1_mop1 --writer-streams 1 --reader-streams 1 --mop 1 &&
run ws32_mop0 --mop 0 &&
run embed_only --mode embed &&
BENCH_PHASE_GAP_MS=5 run ws1_mop1_gap5 --writer-streams 1 --reader-streams 1 --mop 1 &&
cd /tmp && BENCH_PHASE_GAP_MS=5 timeout -k 10 300 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/$O/pgap -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --host-api 0 --writer-streams 1 --reader-streams 1 > $GRAFT_REPO_ROOT/$O/gapprof.json 2>&1 &&
echo done
