# round 3, call 17: device-memory doorbell probe; command ring VRAM request mode (tests + host-API
# A/B); whole GPU test suite; smoke; short bench.py with every row; KV PMC passes.
# A step that fails its checks (rc 1/2) does not stop the call; a fault, abort or time limit does.
set -x
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r3_17
mkdir -p $O
step() { "$@"; rc=$?; case $rc in 0|1|2) return 0;; *) echo "step rc=$rc: stopping"; exit $rc;; esac; }
step timeout -k 10 60 dev/debug/vram_doorbell_probe > $O/probe.jsonl 2> $O/probe.err
SPLINTER_RING_VRAM=1 step timeout -k 10 300 python -u -m pytest tests/test_ring_gpu.py -x -v -m gpu --timeout 120 --timeout-method thread > $O/pytest_ring_vram.log 2>&1
H=libsplinter_amd/bin/splinter_hostapi_bench
for v in 0 1; do for t in 1 16 32; do SPLINTER_RING_VRAM=$v step timeout -k 10 60 $H --threads $t --seconds 1.5 --keys 20000 >> $O/hostapi_vram$v.jsonl 2>> $O/hostapi.err; done; done
step timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1
step timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1
step timeout -k 10 400 python bench.py --keys-per-gpu 10000000 --search-keys 2000000 --steps 5 --warmup 2 --embed-e2e 3 --daemon-docs 256 --routed-steps 3 > $O/bench_small.json 2> $O/bench_small.err
K="--mode kv --host-api 0 --host-api-threads2 0 --routed-steps 0 --steps 4 --warmup 1"
P="rocprofv3 --kernel-trace --output-format csv"
step timeout -s KILL 300 $P --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum -d $O/pmc -o kv_l2 -- python3 bench.py $K > $O/kv_l2.log 2>&1
step timeout -s KILL 300 $P --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VMEM GRBM_GUI_ACTIVE -d $O/pmc -o kv_sq -- python3 bench.py $K > $O/kv_sq.log 2>&1
find $O -name "*kernel_trace.csv" -size +60M -delete
echo done
