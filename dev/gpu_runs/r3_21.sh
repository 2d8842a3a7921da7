# round 3, call 21: where do the set kernel's ~52 EA write requests per op come from?  KV-only A/B
# (default coop carry kernel / per-lane copy / write-through rounds) and TCC write-path counters.
set -x
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r3_21
mkdir -p $O
K="--mode kv --host-api 0 --host-api-threads2 0 --routed-steps 0"
timeout -k 10 300 python -u bench.py $K --steps 10 --warmup 2 > $O/kv_default.json 2> $O/kv_default.err || exit 1
SPLINTER_ARENA_COOP=0 timeout -k 10 300 python -u bench.py $K --steps 10 --warmup 2 > $O/kv_coop0.json 2> $O/kv_coop0.err || exit 1
SPLINTER_ARENA_WT=1 timeout -k 10 300 python -u bench.py $K --steps 10 --warmup 2 > $O/kv_wt1.json 2> $O/kv_wt1.err || exit 1
P="rocprofv3 --kernel-trace --output-format csv"
timeout -s KILL 300 $P --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_EA0_ATOMIC_sum TCC_ALL_TC_OP_WB_WRITEBACK_sum -d $O/pmc -o p1 -- python3 bench.py $K --steps 3 --warmup 1 > $O/p1.log 2>&1 || exit 1
timeout -s KILL 300 $P --pmc TCC_NORMAL_WRITEBACK_sum TCC_ATOMIC_sum TCC_WRITE_sum TCC_WRITEBACK_sum -d $O/pmc -o p2 -- python3 bench.py $K --steps 3 --warmup 1 > $O/p2.log 2>&1 || exit 1
SPLINTER_ARENA_WT=1 timeout -s KILL 300 $P --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_EA0_ATOMIC_sum TCC_ALL_TC_OP_WB_WRITEBACK_sum -d $O/pmc -o p1wt -- python3 bench.py $K --steps 3 --warmup 1 > $O/p1wt.log 2>&1 || exit 1
find $O -name "*kernel_trace.csv" -delete
echo done
