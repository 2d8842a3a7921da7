# round 2, call 3: 32 writer / 32 reader streams at larger per-stream batches
set -x
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r2_03
mkdir -p $O
run() { tag=$1; shift; timeout -k 10 200 python bench.py --mode kv "$@" > $O/$tag.json 2> $O/$tag.err; }
run ws32_b32m --batch 32000000 &&
run ws32_b64m --batch 64000000 &&
run ws16_b32m --batch 32000000 --writer-streams 16 --reader-streams 16 &&
run ws32_rs4_b32m --batch 32000000 --reader-streams 4 &&
echo done
