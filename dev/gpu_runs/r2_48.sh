# round 2, call 48: host submission throttle A/B on the mixed step (32 + 32 streams), interleaved
set -x
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r2_48
mkdir -p $O
for t in 0 1 0 1; do timeout -k 10 200 python bench.py --host-api 0 --embed-e2e 0 --throttle $t >> $O/ab.jsonl 2>> $O/ab.err || exit 1; done &&
echo done
