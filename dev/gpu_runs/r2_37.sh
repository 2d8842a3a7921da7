# round 2, call 37: LN fold v2 (vector fold loads, DPP row sums) -- numerics, epilogue A/B, embed A/B
set -x
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r2_37
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_nomic_gpu.py -x -v --timeout 240 --timeout-method thread -k "fold or encoder" > $O/nomic_tests.log 2>&1 &&
timeout -k 10 200 python scripts/gemm_epi_bench.py > $O/epi_ab.jsonl 2> $O/epi_ab.err &&
timeout -k 10 200 python bench.py --mode embed --host-api 0 > $O/embed_fold.json 2> $O/embed_fold.err &&
NOMIC_LN_FOLD=0 timeout -k 10 200 python bench.py --mode embed --host-api 0 > $O/embed_nofold.json 2> $O/embed_nofold.err &&
echo done
