# round 2, call 2: KV-only A/B of writer/reader stream counts, scrub mode and ops-per-lane
set -x
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r2_02
mkdir -p $O
run() { tag=$1; shift; timeout -k 10 200 python bench.py --mode kv "$@" > $O/$tag.json 2> $O/$tag.err; }
run ws32_mop0 --mop 0 &&
run ws1_mop1 --writer-streams 1 --reader-streams 1 &&
run ws4_mop1 --writer-streams 4 --reader-streams 4 &&
run ws8_mop1 --writer-streams 8 --reader-streams 8 &&
SPLINTER_ARENA_U=2 run ws32_u2 &&
SPLINTER_ARENA_UGET=4 run ws32_uget4 &&
run ws32_mop1 &&
echo done
