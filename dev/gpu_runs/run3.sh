set -x
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -m pytest tests/test_arena_gpu.py -q > gpurun_out/pytest_arena3.log 2>&1; echo "arena rc=$?"
timeout -k 10 600 python -m pytest tests/test_nomic_gpu.py -q -x > gpurun_out/pytest_nomic3.log 2>&1; echo "nomic rc=$?"
for mo in 0 1 2; do
  SPLINTER_ARENA_MO=$mo timeout -k 10 240 python scripts/kv_micro.py --keys 100000000 --batch 4000000 >> gpurun_out/kv_micro3.log 2>&1 || break
done
echo done
