# round 3, call 43: timed-region kernel traces of the default mixed step and of embed-only with the session-2
# defaults (U=2 sets, acquire-free gets, peeled asm-DMA 256^2 GEMM, k_attn3)
set -x
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r3_43
mkdir -p $O
export SPL_PROFILE_TIMED=1
timeout -s KILL 400 rocprofv3 --kernel-trace --output-format csv -d $O/trace_mixed -o mixed -- python3 bench.py --steps 5 --warmup 3 --host-api 0 --host-api-threads2 0 --embed-e2e 0 --daemon-docs 0 --routed-steps 0 --search-batches 2 > $O/trace_mixed.json 2> $O/trace_mixed.err || exit 1
timeout -s KILL 300 rocprofv3 --kernel-trace --output-format csv -d $O/trace_embed -o embed -- python3 bench.py --mode embed --host-api 0 --host-api-threads2 0 --embed-e2e 0 --daemon-docs 0 --steps 6 --warmup 2 --keys-per-gpu 1000000 --search-keys 0 > $O/trace_embed.json 2> $O/trace_embed.err || exit 1
unset SPL_PROFILE_TIMED
T=$(find $O/trace_mixed -name "*kernel_trace.csv" | head -1)
python3 scripts/trace_window.py $T $O/trace_mixed.err --md $O/trace_mixed.md --timeline || exit 1
T=$(find $O/trace_embed -name "*kernel_trace.csv" | head -1)
python3 scripts/trace_window.py $T $O/trace_embed.err --md $O/trace_embed.md || exit 1
find $O -name "*_trace.csv" -delete
echo done
