# round 2, call 22: post-KV embed slowdown vs link order of the HIP objects
set -x
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r2_22
mkdir -p $O
B="--writer-streams 1 --reader-streams 1 --mop 1 --host-api 0"
for v in ordA ordB default; do
  if [ $v = default ]; then unset SPLINTER_HIP_VARIANT; else export SPLINTER_HIP_VARIANT=$v; fi
  timeout -k 10 200 python bench.py $B > $O/$v.json 2> $O/$v.err || exit 1
done
echo done
