# round 3, call 15: device-memory doorbell probe (host BAR writes, stale-L2 check); the command ring's
# VRAM request mode (SPLINTER_RING_VRAM=1): ring GPU tests + host-API sweep against the host mode
set -x
cd $GRAFT_REPO_ROOT
O=gpurun_out/r3_15
mkdir -p $O
timeout -k 10 60 dev/debug/vram_doorbell_probe > $O/probe.jsonl 2> $O/probe.err || exit 1
SPLINTER_RING_VRAM=1 timeout -k 10 300 python -u -m pytest tests/test_ring_gpu.py -x -v -m gpu --timeout 120 --timeout-method thread > $O/pytest_ring_vram.log 2>&1 || exit 1
H=libsplinter_amd/bin/splinter_hostapi_bench
for v in 0 1; do for t in 1 8 16 24 32; do SPLINTER_RING_VRAM=$v timeout -k 10 60 $H --threads $t --seconds 1.5 --keys 20000 | sed "s/^{/{\"vram\": $v, /" >> $O/hostapi.jsonl 2>> $O/hostapi.err || exit 1; done; done
echo done
