# round 3, call 34: where the routed step's extra time goes at N=1 (the N>1 bench path): bench
# --force-routed without and with a timed-region kernel trace
set -x
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r3_34
mkdir -p $O
R="--force-routed --host-api 0 --host-api-threads2 0 --embed-e2e 0 --daemon-docs 0 --search-batches 2"
timeout -k 10 300 python3 -u bench.py $R --steps 20 --warmup 5 > $O/routed.json 2> $O/routed.err || exit 1
timeout -k 10 300 python3 -u bench.py $R --mode kv --steps 10 --warmup 3 > $O/routed_kv.json 2> $O/routed_kv.err || exit 1
export SPL_PROFILE_TIMED=1
timeout -s KILL 400 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/trace_routed -o routed -- python3 bench.py $R --steps 5 --warmup 3 > $O/trace_routed.json 2> $O/trace_routed.err || exit 1
unset SPL_PROFILE_TIMED
T=$(find $O/trace_routed -name "*kernel_trace.csv" | head -1)
python3 scripts/trace_window.py $T $O/trace_routed.err --md $O/trace_routed.md --csv $O/trace_routed.csv --timeline || exit 1
find $O -name "*_trace.csv" -size +60M -delete
echo done
