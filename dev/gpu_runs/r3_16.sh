# round 3, call 16: whole GPU test suite, smoke, and a short bench.py with every row (daemon path included)
set -x
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r3_16
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 400 python bench.py --keys-per-gpu 10000000 --search-keys 2000000 --steps 5 --warmup 2 --embed-e2e 3 --daemon-docs 256 --routed-steps 3 > $O/bench_small.json 2> $O/bench_small.err || exit 1
echo done
K="--mode kv --host-api 0 --host-api-threads2 0 --routed-steps 0 --steps 4 --warmup 1"
P="rocprofv3 --kernel-trace --output-format csv"
timeout -s KILL 300 $P --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum -d $O/pmc -o kv_l2 -- python3 bench.py $K > $O/kv_l2.log 2>&1 &&
timeout -s KILL 300 $P --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VMEM GRBM_GUI_ACTIVE -d $O/pmc -o kv_sq -- python3 bench.py $K > $O/kv_sq.log 2>&1 &&
find $O -name "*kernel_trace.csv" -size +60M -delete ; echo done2
