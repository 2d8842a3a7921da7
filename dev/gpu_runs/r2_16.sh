# round 2, call 16: post-KV embed slowdown -- copies in the step? TLB / L2 counters of k_ln (old vs new)
set -x
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r2_16
mkdir -p $O
cd /tmp
B="--steps 5 --warmup 2 --writer-streams 1 --reader-streams 1 --mop 0 --host-api 0"
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d $O/tnew -o run -- python3 $GRAFT_REPO_ROOT/bench.py $B > $O/tnew.json 2> $O/tnew.err &&
timeout -s KILL 200 rocprofv3 --pmc TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCC_HIT_sum TCC_MISS_sum --kernel-include-regex "k_ln|k_gemm_nt" -d $O/cnew -o run -- python3 $GRAFT_REPO_ROOT/bench.py $B > $O/cnew.json 2> $O/cnew.err &&
timeout -s KILL 200 rocprofv3 --pmc TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCC_HIT_sum TCC_MISS_sum --kernel-include-regex "k_ln|k_gemm_nt" -d $O/cold -o run -- python3 $GRAFT_REPO_ROOT/ab_old/bench.py --steps 5 --warmup 2 > $O/cold.json 2> $O/cold.err &&
echo done
