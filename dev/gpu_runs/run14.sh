# PMC counters (each run: --pmc + kernel-trace only): MFMA / LDS for GEMM + attention, cache/atomics for KV
set -x
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc14
P="rocprofv3 --kernel-trace --output-format csv"
timeout -k 10 300 $P --pmc SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d gpurun_out/pmc14 -o gemm_mfma -- python3 scripts/gemm_bench.py --tokens 65536 --rounds 1 --iters 2 > gpurun_out/pmc14/gemm_mfma.log 2>&1 &&
timeout -k 10 300 $P --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES -d gpurun_out/pmc14 -o gemm_lds -- python3 scripts/gemm_bench.py --tokens 65536 --rounds 1 --iters 2 > gpurun_out/pmc14/gemm_lds.log 2>&1 &&
timeout -k 10 300 $P --pmc SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d gpurun_out/pmc14 -o attn_mfma -- python3 scripts/attn_bench.py --docs 64 --rounds 1 --iters 2 > gpurun_out/pmc14/attn_mfma.log 2>&1 &&
timeout -k 10 300 $P --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES -d gpurun_out/pmc14 -o attn_lds -- python3 scripts/attn_bench.py --docs 64 --rounds 1 --iters 2 > gpurun_out/pmc14/attn_lds.log 2>&1 &&
timeout -k 10 300 $P --pmc TCC_EA0_ATOMIC_sum TCC_EA0_ATOMIC_LEVEL_sum TCC_ALL_TC_OP_WB_WRITEBACK_sum TCC_ALL_TC_OP_INV_EVICT_sum -d gpurun_out/pmc14 -o kv_atomic -- python3 scripts/kv_micro.py --keys 20000000 --batch 8000000 --reps 2 > gpurun_out/pmc14/kv_atomic.log 2>&1 &&
timeout -k 10 300 $P --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum -d gpurun_out/pmc14 -o kv_cache -- python3 scripts/kv_micro.py --keys 20000000 --batch 8000000 --reps 2 > gpurun_out/pmc14/kv_cache.log 2>&1 &&
echo done
