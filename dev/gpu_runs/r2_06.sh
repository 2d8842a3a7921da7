# round 2, call 6: native 64-stream fan-out (kv_streams.hip) in the headline bench
set -x
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r2_06
mkdir -p $O
run() { tag=$1; shift; timeout -k 10 200 python bench.py "$@" > $O/$tag.json 2> $O/$tag.err; }
run kv --mode kv --host-api 0 &&
run mixed &&
run mixed_ws1 --writer-streams 1 --reader-streams 1 --host-api 0 &&
echo done
