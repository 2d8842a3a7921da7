# round 3, call 46: where a batched search (config #5, 25M x 768 per GPU) spends its time: kernel stats
set -x
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r3_46
mkdir -p $O
timeout -k 10 300 python3 -u scripts/search_bench.py --slots 25000000 --nq 512 --iters 3 > $O/search.json 2> $O/search.err || exit 1
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o search -- python3 scripts/search_bench.py --slots 25000000 --nq 512 --iters 3 > $O/trace.json 2> $O/trace.err || exit 1
find $O -name "*kernel_trace.csv" -delete
echo done
