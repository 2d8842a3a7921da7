# rounds kernels: block-size / per-op-kind U sweep
set -x
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_arena_gpu.py -q -x > gpurun_out/pytest_arena12.log 2>&1 &&
timeout -k 10 300 python scripts/kv_micro.py --batch 8000000 > gpurun_out/kv12_default.log 2>&1 &&
SPLINTER_ARENA_BLOCK=512 timeout -k 10 300 python scripts/kv_micro.py --batch 8000000 > gpurun_out/kv12_b512.log 2>&1 &&
SPLINTER_ARENA_BLOCK=512 SPLINTER_ARENA_U=2 SPLINTER_ARENA_UGET=2 timeout -k 10 300 python scripts/kv_micro.py --batch 8000000 > gpurun_out/kv12_b512_u2.log 2>&1 &&
SPLINTER_ARENA_UGET=4 timeout -k 10 300 python scripts/kv_micro.py --batch 8000000 > gpurun_out/kv12_u4u4.log 2>&1 &&
timeout -k 10 400 python bench.py --mode kv > gpurun_out/bench12_kv.log 2>&1 &&
SPLINTER_ARENA_BLOCK=512 timeout -k 10 400 python bench.py --mode kv > gpurun_out/bench12_kv_b512.log 2>&1 &&
timeout -k 10 400 python bench.py > gpurun_out/bench12.log 2>&1 &&
echo done
