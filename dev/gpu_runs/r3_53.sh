# round 3, call 53: cheap knobs -- L2 band width of the 256^2 GEMM tile order (NOMIC_GEMM_GN) on the embed step;
# 3 hardware queues per priority on the mixed step
set -x
cd $GRAFT_REPO_ROOT
O=gpurun_out/r3_53
mkdir -p $O
E="--mode embed --embed-e2e 0 --daemon-docs 0 --host-api 0 --host-api-threads2 0 --routed-steps 0 --steps 20 --warmup 5"
M="--mode mixed --embed-e2e 0 --daemon-docs 0 --search-batches 2 --host-api 0 --host-api-threads2 0 --routed-steps 0 --steps 20 --warmup 5"
run() { tag=$1; shift; e=(); while [[ $1 == *=* ]]; do e+=("$1"); shift; done; env "${e[@]}" timeout -k 10 300 python -u bench.py "$@" 2>> $O/b.err | sed "s/^{/{\"tag\": \"$tag\", /" >> $O/ab.jsonl; }
for r in 1 2; do
run embed_gn_default X=1 $E || exit 1
run embed_gn2 NOMIC_GEMM_GN=2 $E || exit 1
run embed_gn3 NOMIC_GEMM_GN=3 $E || exit 1
run embed_gn6 NOMIC_GEMM_GN=6 $E || exit 1
run embed_gn8 NOMIC_GEMM_GN=8 $E || exit 1
done
for r in 1 2; do
run mixed_q2 X=1 $M || exit 1
run mixed_q3 SPLINTER_BENCH_HW_QUEUES=3 $M || exit 1
done
echo done
