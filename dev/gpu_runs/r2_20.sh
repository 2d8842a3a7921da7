# round 2, call 20: bisect the post-KV embed slowdown -- lib without the ring / fan-out objects
set -x
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r2_20
mkdir -p $O
B="--writer-streams 1 --reader-streams 1 --mop 1 --host-api 0"
SPLINTER_HBM_NO_RING=1 BENCH_SKIP_MOP=1 BENCH_PY_STREAMS=1 SPLINTER_HIP_VARIANT=noringobj timeout -k 10 200 python bench.py $B > $O/noringobj.json 2> $O/noringobj.err &&
BENCH_SKIP_MOP=1 BENCH_PY_STREAMS=1 timeout -k 10 200 python bench.py $B > $O/new.json 2> $O/new.err &&
echo done
