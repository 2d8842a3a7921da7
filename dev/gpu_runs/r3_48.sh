# round 3, call 48: end-of-session validation -- full GPU suite, smoke, bench with driver arguments (twice),
# 2-rank gloo rehearsal of the routed (N>1) step on one GPU
set -x
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r3_48
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit 1
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || exit 1
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > $O/bench2.json 2> $O/bench2.err || exit 1
timeout -k 10 400 python bench.py --gpus 2 --backend gloo --keys-per-gpu 2000000 --batch 1000000 --embed-batch 8 --steps 3 --warmup 1 --host-api 0 --embed-e2e 2 > $O/gloo2.json 2> $O/gloo2.err || exit 1
echo done
