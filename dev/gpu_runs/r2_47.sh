# round 2, call 47: PMC of the encoder forward (MFMA busy per kernel) in the embed bench -- counters only with kernel-trace
set -x
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r2_47
mkdir -p $O
P="rocprofv3 --kernel-trace --output-format csv"
timeout -k 10 300 $P --pmc SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $O/pmc -o enc_mfma -- python3 bench.py --mode embed --host-api 0 --embed-e2e 0 --steps 3 --warmup 1 --keys-per-gpu 1000000 > $O/enc_mfma.log 2>&1 &&
timeout -k 10 300 $P --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS -d $O/pmc -o enc_lds -- python3 bench.py --mode embed --host-api 0 --embed-e2e 0 --steps 3 --warmup 1 --keys-per-gpu 1000000 > $O/enc_lds.log 2>&1 &&
echo done
