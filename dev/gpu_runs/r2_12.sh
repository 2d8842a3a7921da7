# round 2, call 12: bisect the slower post-KV embed phase (device-header bus probe in from_api)
set -x
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r2_12
mkdir -p $O
B="--writer-streams 1 --reader-streams 1 --mop 0 --host-api 0"
SPLINTER_HIP_VARIANT=noprobe timeout -k 10 200 python bench.py $B > $O/noprobe.json 2> $O/noprobe.err &&
timeout -k 10 200 python bench.py $B > $O/probe.json 2> $O/probe.err &&
SPLINTER_HIP_VARIANT=noprobe timeout -k 10 200 python bench.py $B > $O/noprobe2.json 2> $O/noprobe2.err &&
echo done
