# round 2, call 40: splainference on HIP -- causal prefill attention, GEMV decode step, device sampler, graph replay
set -x
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r2_40
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_splainference.py -x -v -s --timeout 200 --timeout-method thread > $O/tests.log 2>&1 &&
timeout -k 10 200 python -u -m pytest tests/test_nomic_gpu.py -x -q --timeout 150 --timeout-method thread -k "attention or encoder" > $O/nomic.log 2>&1 &&
echo done
