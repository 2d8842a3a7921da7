# round 3, call 18: VRAM-mode ring with one-store completions: ring tests, TAP suites on hbm:/node:,
# host-API sweep and the oversubscribed sleep length A/B
set -x
cd $GRAFT_REPO_ROOT
O=gpurun_out/r3_18
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_ring_gpu.py tests/test_node_gpu.py tests/test_arena_gpu.py -x -v -m gpu --timeout 150 --timeout-method thread > $O/pytest_ring.log 2>&1 || exit 1
H=libsplinter_amd/bin/splinter_hostapi_bench
for t in 1 8 16 24 32; do timeout -k 10 60 $H --threads $t --seconds 1.5 --keys 20000 >> $O/hostapi.jsonl 2>> $O/hostapi.err || exit 1; done
for ns in 1000 5000; do for t in 24 32; do SPLINTER_RING_SLEEP_NS=$ns timeout -k 10 60 $H --threads $t --seconds 1.5 --keys 20000 | sed "s/^{/{\"sleep_ns\": $ns, /" >> $O/hostapi_sleep.jsonl 2>> $O/hostapi.err || exit 1; done; done
for t in 16 32; do SPLINTER_RING_VRAM=0 timeout -k 10 60 $H --threads $t --seconds 1.5 --keys 20000 | sed "s/^{/{\"vram\": 0, /" >> $O/hostapi_host.jsonl 2>> $O/hostapi.err || exit 1; done
echo done
