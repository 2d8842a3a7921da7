set -x
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_arena_gpu.py -q -x > gpurun_out/pytest_arena19.log 2>&1 &&
timeout -k 10 300 python scripts/kv_micro.py --batch 8000000 > gpurun_out/kv19_copy1.log 2>&1 &&
SPLINTER_ARENA_GETCOPY=2 timeout -k 10 300 python scripts/kv_micro.py --batch 8000000 > gpurun_out/kv19_copy2.log 2>&1 &&
timeout -k 10 400 python bench.py --mode kv > gpurun_out/bench19_kv.log 2>&1 &&
echo done
