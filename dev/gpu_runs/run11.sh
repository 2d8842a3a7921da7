# workgroup-aggregated fences: arena tests, then U sweep micro + kv bench
set -x
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_arena_gpu.py tests/test_search_gpu.py -q -x > gpurun_out/pytest_arena11.log 2>&1 &&
SPLINTER_ARENA_U=4 timeout -k 10 300 python scripts/kv_micro.py --batch 8000000 > gpurun_out/kv11_u4.log 2>&1 &&
SPLINTER_ARENA_U=8 timeout -k 10 300 python scripts/kv_micro.py --batch 8000000 > gpurun_out/kv11_u8.log 2>&1 &&
SPLINTER_ARENA_U=2 timeout -k 10 300 python scripts/kv_micro.py --batch 8000000 > gpurun_out/kv11_u2.log 2>&1 &&
timeout -k 10 400 python bench.py --mode kv > gpurun_out/bench11_kv.log 2>&1 &&
SPLINTER_ARENA_U=8 timeout -k 10 400 python bench.py --mode kv > gpurun_out/bench11_kv_u8.log 2>&1 &&
echo done
