# round 3, call 56: final validation of the tree -- full GPU suite, smoke, bench with driver arguments
set -x
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r3_56
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit 1
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || exit 1
timeout -k 10 300 python -u scripts/decode_q4_bench.py --layers 8 --rounds 2 > $O/dec.jsonl 2> $O/dec.err || exit 1
echo done
