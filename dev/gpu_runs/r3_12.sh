# round 3, call 12: full kernel traces of bench.py (embed mode and the default mixed step) with the
# timed region's clock bounds (SPL_PROFILE_TIMED=1) -> scripts/trace_window.py; bench.py embed mode
set -x
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r3_12
mkdir -p $O
export SPL_PROFILE_TIMED=1
timeout -s KILL 300 rocprofv3 --kernel-trace --output-format csv -d $O/trace_embed -o embed -- python3 bench.py --mode embed --host-api 0 --host-api-threads2 0 --embed-e2e 0 --steps 6 --warmup 2 --keys-per-gpu 1000000 --search-keys 0 > $O/trace_embed.json 2> $O/trace_embed.err &&
timeout -s KILL 600 rocprofv3 --kernel-trace --output-format csv -d $O/trace_mixed -o mixed -- python3 bench.py --steps 5 --warmup 3 --host-api 0 --host-api-threads2 0 --embed-e2e 0 --routed-steps 0 --search-batches 2 > $O/trace_mixed.json 2> $O/trace_mixed.err &&
unset SPL_PROFILE_TIMED &&
timeout -k 10 300 python bench.py --mode embed --host-api 0 --host-api-threads2 0 --embed-e2e 10 --steps 20 --warmup 3 --keys-per-gpu 1000000 --search-keys 0 > $O/bench_embed.json 2> $O/bench_embed.err &&
find $O -name "*kernel_trace.csv" -size +60M -delete ; echo done
