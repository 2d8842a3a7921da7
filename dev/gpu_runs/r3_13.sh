# round 3, call 13: 32x32-MFMA attention (k_attn3) numerics + A/B; host-API ring, every waiter sleep-polls while oversubscribed (A/B on the CPU threshold)
set -x
cd $GRAFT_REPO_ROOT
O=gpurun_out/r3_13
mkdir -p $O
H=libsplinter_amd/bin/splinter_hostapi_bench
for t in 1 16 24 32 48; do timeout -k 10 60 $H --threads $t --seconds 1.5 --keys 20000 >> $O/hostapi_default.jsonl 2>> $O/hostapi.err || exit 1; done
for c in 8 12; do for t in 16 32; do SPLINTER_RING_CPUS=$c timeout -k 10 60 $H --threads $t --seconds 1.5 --keys 20000 | sed "s/^{/{\"ring_cpus\": $c, /" >> $O/hostapi_cpus.jsonl 2>> $O/hostapi.err || exit 1; done; done
echo done
timeout -k 10 200 python -u -m pytest tests/test_nomic_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread -k "attention_varlen" > $O/pytest_attn.log 2>&1 || exit 1
ATTN_VARIANTS=6,13 timeout -k 10 200 python -u scripts/attn_bench.py --rounds 7 > $O/attn_ab.jsonl 2> $O/attn_ab.err || exit 1
echo done2
