# round 3, call 36: where the encoder kernels' wave cycles go (SQ stall counters), lockstep vs ping-pong
# 256^2 GEMM; MFMA busy of the shipped kernels (k_attn3 now the default attention)
set -x
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r3_36
mkdir -p $O
B="--mode embed --host-api 0 --host-api-threads2 0 --embed-e2e 0 --daemon-docs 0 --routed-steps 0 --steps 3 --warmup 1 --keys-per-gpu 1000000 --search-keys 0"
P="rocprofv3 --kernel-trace --output-format csv"
S="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE"
timeout -s KILL 240 $P --pmc $S -d $O/pmc -o sq_pp0 -- python3 bench.py $B > $O/sq_pp0.log 2>&1 || exit 1
NOMIC_GEMM_PP=1 timeout -s KILL 240 $P --pmc $S -d $O/pmc -o sq_pp1 -- python3 bench.py $B > $O/sq_pp1.log 2>&1 || exit 1
timeout -s KILL 240 $P --pmc SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $O/pmc -o enc_mfma -- python3 bench.py $B > $O/enc_mfma.log 2>&1 || exit 1
timeout -s KILL 240 $P --pmc TCC_HIT_sum TCC_MISS_sum SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE -d $O/pmc -o enc_l2 -- python3 bench.py $B > $O/enc_l2.log 2>&1 || exit 1
find $O -name "*kernel_trace.csv" -delete
echo done
