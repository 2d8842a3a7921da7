set -x
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -m gpu -q > gpurun_out/pytest_gpu5.log 2>&1; echo "pytest rc=$?"
for u in 1 2 4 8; do
  SPLINTER_ARENA_U=$u timeout -k 10 240 python scripts/kv_micro.py --keys 100000000 --batch 4000000 >> gpurun_out/kv_micro5.log 2>&1
done
echo done
