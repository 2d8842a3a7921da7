# round 2, call 36: LN folded into the encoder GEMMs -- numerics, then embed A/B (fold on/off) and a kernel profile
set -x
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r2_36
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_nomic_gpu.py -x -v --timeout 300 --timeout-method thread > $O/nomic_tests.log 2>&1 &&
timeout -k 10 200 python bench.py --mode embed --host-api 0 > $O/embed_fold.json 2> $O/embed_fold.err &&
NOMIC_LN_FOLD=0 timeout -k 10 200 python bench.py --mode embed --host-api 0 > $O/embed_nofold.json 2> $O/embed_nofold.err &&
timeout -k 10 200 python bench.py --mode embed --host-api 0 > $O/embed_fold2.json 2> $O/embed_fold2.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o embed -- python bench.py --mode embed --host-api 0 --steps 10 > $O/prof.log 2>&1 &&
echo done
