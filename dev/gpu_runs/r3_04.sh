# round 3, call 4: interleaved-load variants of the residual+LN kernel (numerics + A/B + PMC), node-store GPU tests
set -x
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r3_04
mkdir -p $O
for v in 210 220 230; do NOMIC_RLN=$v timeout -k 10 120 python -u -m pytest tests/test_nomic_gpu.py -x -q --timeout 60 --timeout-method thread -k "residual_layernorm" > $O/pytest_v$v.log 2>&1 || exit 1; done
timeout -k 10 300 python scripts/residual_gemm_ab.py --rln-variants 10,20,30,210,220,230 > $O/rln_ab.jsonl 2> $O/rln_ab.err || exit 1
timeout -k 10 300 python -u -m pytest tests/test_node_gpu.py -v --timeout 120 --timeout-method thread > $O/pytest_node.log 2>&1
echo "node tests rc=$?"
P2=SQ_LDS_BANK_CONFLICT,SQ_LDS_IDX_ACTIVE,SQ_WAVE_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,SQ_WAIT_INST_LDS,SQ_INSTS_VALU
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc $P2 --kernel-trace -d $GRAFT_REPO_ROOT/$O/pmc2_v220 -o run -- python3 $GRAFT_REPO_ROOT/scripts/rln_pmc.py --impl v220 > /dev/null 2>&1 || exit 1
echo done
