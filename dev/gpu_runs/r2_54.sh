# round 2, call 54: ops per lane of the seqlock kernels for the 32 + 32-stream fan-out (250K-op batches per stream)
set -x
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r2_54
mkdir -p $O
for cfg in "4 2" "1 1" "2 1" "1 2" "4 2"; do set -- $cfg; SPLINTER_ARENA_U=$1 SPLINTER_ARENA_UGET=$2 timeout -k 10 200 python bench.py --mode kv --host-api 0 --embed-e2e 0 | sed "s/^{/{\"u\": $1, \"uget\": $2, /" >> $O/kv.jsonl 2>> $O/kv.err || exit 1; done &&
echo done
