# round 3, call 19: VRAM-mode ring with one-store completions (ring / node / arena GPU tests, TAP on
# hbm:/node:), host-API sweep + sleep-length A/B; attention variants 13-15 (3 waves/SIMD, 2-tile prefetch)
set -x
cd $GRAFT_REPO_ROOT
O=gpurun_out/r3_19
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_ring_gpu.py tests/test_node_gpu.py tests/test_arena_gpu.py -x -v -m gpu --timeout 150 --timeout-method thread > $O/pytest_ring.log 2>&1 || exit 1
H=libsplinter_amd/bin/splinter_hostapi_bench
for t in 1 8 16 24 32; do timeout -k 10 60 $H --threads $t --seconds 1.5 --keys 20000 >> $O/hostapi.jsonl 2>> $O/hostapi.err || exit 1; done
for ns in 1000 5000; do for t in 24 32; do SPLINTER_RING_SLEEP_NS=$ns timeout -k 10 60 $H --threads $t --seconds 1.5 --keys 20000 | sed "s/^{/{\"sleep_ns\": $ns, /" >> $O/hostapi_sleep.jsonl 2>> $O/hostapi.err || exit 1; done; done
for t in 16 32; do SPLINTER_RING_VRAM=0 timeout -k 10 60 $H --threads $t --seconds 1.5 --keys 20000 | sed "s/^{/{\"vram\": 0, /" >> $O/hostapi_host.jsonl 2>> $O/hostapi.err || exit 1; done
timeout -k 10 200 python -u -m pytest tests/test_nomic_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread -k "attention_varlen" > $O/pytest_attn.log 2>&1 || exit 1
ATTN_VARIANTS=6,13,14,15 timeout -k 10 200 python -u scripts/attn_bench.py --rounds 7 > $O/attn_ab.jsonl 2> $O/attn_ab.err || exit 1
echo done
