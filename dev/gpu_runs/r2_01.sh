# round 2, call 1: GPU suite + smoke, headline bench (32 writer / 32 reader streams, hybrid mop),
# A/B against the round-1 config (2 streams, mop 0), the --gpus 2 launcher (gloo rehearsal) and
# a kernel-trace profile of the default bench
set -x
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r2_01
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 &&
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 &&
timeout -k 10 300 python bench.py > $O/bench_default.json 2> $O/bench_default.err &&
timeout -k 10 300 python bench.py --writer-streams 1 --reader-streams 1 --mop 0 > $O/bench_r1cfg.json 2> $O/bench_r1cfg.err &&
timeout -k 10 300 python bench.py --mode kv > $O/bench_kv.json 2> $O/bench_kv.err &&
timeout -k 10 300 python bench.py --gpus 2 --backend gloo --keys-per-gpu 1000000 --batch 1000000 --mode kv --steps 3 --warmup 1 > $O/bench_gloo2.json 2> $O/bench_gloo2.err &&
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 > $GRAFT_REPO_ROOT/$O/bench_prof.json 2> $GRAFT_REPO_ROOT/$O/bench_prof.err &&
echo done
