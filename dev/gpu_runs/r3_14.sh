# round 3, call 14: host-API ring sweep (every waiter sleep-polls while oversubscribed); full kernel
# traces of bench.py embed / mixed with the timed-region bounds; 32x32-MFMA attention (k_attn3)
set -x
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r3_14
mkdir -p $O
H=libsplinter_amd/bin/splinter_hostapi_bench
for t in 1 16 24 32 48; do timeout -k 10 60 $H --threads $t --seconds 1.5 --keys 20000 >> $O/hostapi_default.jsonl 2>> $O/hostapi.err || exit 1; done
for c in 8 12; do for t in 16 32; do SPLINTER_RING_CPUS=$c timeout -k 10 60 $H --threads $t --seconds 1.5 --keys 20000 | sed "s/^{/{\"ring_cpus\": $c, /" >> $O/hostapi_cpus.jsonl 2>> $O/hostapi.err || exit 1; done; done
export SPL_PROFILE_TIMED=1
timeout -s KILL 300 rocprofv3 --kernel-trace --output-format csv -d $O/trace_embed -o embed -- python3 bench.py --mode embed --host-api 0 --host-api-threads2 0 --embed-e2e 0 --steps 6 --warmup 2 --keys-per-gpu 1000000 --search-keys 0 > $O/trace_embed.json 2> $O/trace_embed.err || exit 1
timeout -s KILL 600 rocprofv3 --kernel-trace --output-format csv -d $O/trace_mixed -o mixed -- python3 bench.py --steps 5 --warmup 3 --host-api 0 --host-api-threads2 0 --embed-e2e 0 --routed-steps 0 --search-batches 2 > $O/trace_mixed.json 2> $O/trace_mixed.err || exit 1
unset SPL_PROFILE_TIMED
find $O -name "*kernel_trace.csv" -size +60M -delete
timeout -k 10 200 python -u -m pytest tests/test_nomic_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread -k "attention_varlen" > $O/pytest_attn.log 2>&1 || exit 1
ATTN_VARIANTS=6,13 timeout -k 10 200 python -u scripts/attn_bench.py --rounds 7 > $O/attn_ab.jsonl 2> $O/attn_ab.err || exit 1
echo done
