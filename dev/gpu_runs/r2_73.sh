# round 2, call 73: pipelined e2e embedding (side-stream fetch, pinned async Batch upload, daemon lookahead)
# A/B against the previous tree (ab_old/), GPU tests of the touched paths, kernel trace of the q4 decode step
set -x
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r2_73
mkdir -p $O
B="--mode embed --host-api 0 --embed-e2e 20 --steps 10"
timeout -k 10 600 python -u -m pytest tests/test_nomic_gpu.py tests/test_search_gpu.py tests/test_splainference.py -x -v --timeout 200 --timeout-method thread -m gpu > $O/tests.log 2>&1 &&
for t in new old new old; do
  if [ $t = new ]; then d=$GRAFT_REPO_ROOT; else d=$GRAFT_REPO_ROOT/ab_old; fi
  (cd $d && timeout -k 10 200 python bench.py $B --keys-per-gpu 1000000) | sed "s/^{/{\"tree\": \"$t\", /" >> $O/e2e.jsonl 2>> $O/e2e.err || exit 1
done &&
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/prof -o run -- python3 scripts/decode_q4_bench.py --layers 2 --tokens 16 --rounds 1 > $O/dq4.jsonl 2> $O/dq4.err &&
echo done
