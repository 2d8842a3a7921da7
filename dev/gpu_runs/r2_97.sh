# round 2, call 97: hardware queues per priority (SPLINTER_BENCH_HW_QUEUES 3 vs 2) with the writer spread, mixed step
set -x
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r2_97
mkdir -p $O
B="--host-api 0 --embed-e2e 0"
for q in 3 2 3 2; do SPLINTER_BENCH_HW_QUEUES=$q timeout -k 10 200 python bench.py $B | sed "s/^{/{\"hwq\": $q, /" >> $O/mixed.jsonl 2>> $O/mixed.err || exit 1; done &&
echo done
