# round 3, call 40: host-API ring waiting policy while oversubscribed (32 threads on the box's 16-CPU share):
# first sleep length and the initial spin, alternating rounds
set -x
cd $GRAFT_REPO_ROOT
O=gpurun_out/r3_40
mkdir -p $O
H=libsplinter_amd/bin/splinter_hostapi_bench
run() { tag=$1; shift; e=(); while [[ $1 == *=* ]]; do e+=("$1"); shift; done; env "${e[@]}" timeout -k 10 60 $H --threads 32 --seconds 1.5 --keys 20000 "$@" 2>> $O/h.err | sed "s/^{/{\"tag\": \"$tag\", /" >> $O/h.jsonl; }
for r in 1 2 3; do
run base X=1 || exit 1
run first8 SPLINTER_RING_FIRST_SLEEP_NS=8000 || exit 1
run first10 SPLINTER_RING_FIRST_SLEEP_NS=10000 || exit 1
run nospin SPLINTER_RING_OVERSUB_SPIN_US=0 || exit 1
run nospin_first8 SPLINTER_RING_OVERSUB_SPIN_US=0 SPLINTER_RING_FIRST_SLEEP_NS=8000 || exit 1
run sleep3_first8 SPLINTER_RING_SLEEP_NS=3000 SPLINTER_RING_FIRST_SLEEP_NS=8000 || exit 1
done
for t in 1 16; do timeout -k 10 60 $H --threads $t --seconds 1.5 --keys 20000 | sed "s/^{/{\"tag\": \"base_t$t\", /" >> $O/h.jsonl || exit 1; done
echo done
