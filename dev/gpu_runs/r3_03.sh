# round 3, call 3: PMC passes on the residual+LN kernel vs hipBLASLt; 4-wave variants; node-store GPU tests
set -x
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r3_03
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_node_gpu.py -x -v --timeout 120 --timeout-method thread > $O/pytest_node.log 2>&1
echo "node tests rc=$?"
for v in 110 130; do NOMIC_RLN=$v timeout -k 10 120 python -u -m pytest tests/test_nomic_gpu.py -x -q --timeout 60 --timeout-method thread -k "residual_layernorm" > $O/pytest_v$v.log 2>&1 || exit 1; done
timeout -k 10 300 python scripts/residual_gemm_ab.py --rln-variants 10,30,110,130 --no-blas > $O/rln_ab.jsonl 2> $O/rln_ab.err || exit 1
P1=SQ_INSTS_VALU_MFMA_MOPS_BF16,SQ_VALU_MFMA_BUSY_CYCLES,SQ_BUSY_CYCLES,GRBM_GUI_ACTIVE
P2=SQ_LDS_BANK_CONFLICT,SQ_LDS_IDX_ACTIVE,SQ_WAVE_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,SQ_WAIT_INST_LDS,SQ_INSTS_VALU
for impl in v30 blas; do
  cd /tmp
  timeout -s KILL 120 rocprofv3 --pmc $P1 --kernel-trace -d $GRAFT_REPO_ROOT/$O/pmc1_$impl -o run -- python3 $GRAFT_REPO_ROOT/scripts/rln_pmc.py --impl $impl > /dev/null 2>&1 || exit 1
  timeout -s KILL 120 rocprofv3 --pmc $P2 --kernel-trace -d $GRAFT_REPO_ROOT/$O/pmc2_$impl -o run -- python3 $GRAFT_REPO_ROOT/scripts/rln_pmc.py --impl $impl > /dev/null 2>&1 || exit 1
  cd $GRAFT_REPO_ROOT
done
echo done
