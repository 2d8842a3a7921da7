# round 3, call 25: what bounds the KV step -- set-only / get-only runs and a timed-region kernel
# timeline of the KV-only step (union of each kernel's dispatch intervals)
set -x
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r3_25
mkdir -p $O
export SPLINTER_ARENA_COOP_GET=2
K="--mode kv --host-api 0 --host-api-threads2 0 --routed-steps 0 --steps 10 --warmup 2"
for f in 1.0 0.0 0.5; do timeout -k 10 300 python -u bench.py $K --set-frac $f 2>> $O/kv.err | sed "s/^{/{\"set_frac\": $f, /" >> $O/kv_frac.jsonl || exit 1; done
SPL_PROFILE_TIMED=1 timeout -s KILL 300 rocprofv3 --kernel-trace --output-format csv -d $O/tr -o kv -- python3 bench.py $K --steps 5 > $O/kv_trace.json 2> $O/kv_trace.err || exit 1
T=$(find $O/tr -name "kv_kernel_trace.csv" | head -1)
python3 scripts/trace_window.py $T $O/kv_trace.err --timeline --md $O/kv_timeline.md > /dev/null || exit 1
rm -rf $O/tr
echo done
