# round 3, call 39: validation of the new defaults (U=2 sets, acquire-free gets, peeled asm-DMA 256^2 GEMM) --
# full GPU suite, smoke, bench with driver arguments; MFMA-busy PMC pass of the encoder
set -x
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r3_39
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit 1
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || exit 1
B="--mode embed --host-api 0 --host-api-threads2 0 --embed-e2e 0 --daemon-docs 0 --routed-steps 0 --steps 3 --warmup 1 --keys-per-gpu 1000000 --search-keys 0"
timeout -s KILL 240 rocprofv3 --kernel-trace --output-format csv --pmc SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $O/pmc -o enc_mfma -- python3 bench.py $B > $O/enc_mfma.log 2>&1 || exit 1
find $O -name "*kernel_trace.csv" -delete
echo done
