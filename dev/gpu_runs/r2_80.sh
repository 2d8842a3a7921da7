# round 2, call 80: PMC counters of the encoder kernels (MFMA busy, bf16 MFMA ops, LDS conflicts) in bench --mode embed
set -x
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r2_80
mkdir -p $O
B="--mode embed --host-api 0 --embed-e2e 0 --steps 3 --warmup 1 --keys-per-gpu 1000000"
P="rocprofv3 --kernel-trace --output-format csv"
timeout -s KILL 240 $P --pmc SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $O/pmc -o enc_mfma -- python3 bench.py $B > $O/enc_mfma.log 2>&1 &&
timeout -s KILL 240 $P --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_INSTS_VALU -d $O/pmc -o enc_lds -- python3 bench.py $B > $O/enc_lds.log 2>&1 &&
echo done
