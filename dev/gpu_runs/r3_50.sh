# round 3, call 50: host-API ring oversubscribed-wait sweep around the new defaults (32 threads), then a
# 1..48-thread curve; KV PMC pass with the session-2 defaults (U=2 sets, acquire-free gets)
set -x
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r3_50
mkdir -p $O
H=libsplinter_amd/bin/splinter_hostapi_bench
run() { tag=$1; shift; e=(); while [[ $1 == *=* ]]; do e+=("$1"); shift; done; env "${e[@]}" timeout -k 10 60 $H --seconds 1.5 --keys 20000 "$@" 2>> $O/h.err | sed "s/^{/{\"tag\": \"$tag\", /" >> $O/h.jsonl; }
for r in 1 2 3; do
run f8_s5 X=1 --threads 32 || exit 1
run f6_s5 SPLINTER_RING_FIRST_SLEEP_NS=6000 --threads 32 || exit 1
run f10_s5 SPLINTER_RING_FIRST_SLEEP_NS=10000 --threads 32 || exit 1
run f8_s3 SPLINTER_RING_SLEEP_NS=3000 --threads 32 || exit 1
run f8_s8 SPLINTER_RING_SLEEP_NS=8000 --threads 32 || exit 1
done
for t in 1 4 8 16 24 32 40 48; do run curve_t$t X=1 --threads $t || exit 1; done
K="--mode kv --host-api 0 --host-api-threads2 0 --routed-steps 0 --steps 3 --warmup 1"
P="rocprofv3 --kernel-trace --output-format csv"
timeout -s KILL 240 $P --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $O/pmc -o kv_sq -- python3 bench.py $K > $O/kv_sq.log 2>&1 || exit 1
timeout -s KILL 240 $P --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum -d $O/pmc -o kv_l2 -- python3 bench.py $K > $O/kv_l2.log 2>&1 || exit 1
find $O -name "*kernel_trace.csv" -delete
echo done
