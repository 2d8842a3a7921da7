# round 2, call 62: which v3 change costs throughput at 16-24 host threads: v3 vs v3 with the
# staged (v2-order) get vs v3 with the staged set vs v2
set -x
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r2_62
mkdir -p $O
T=libsplinter_amd/bin/splinter_hostapi_bench
L=$PWD/libsplinter_amd/lib
for rep in 1 2; do for th in 1 16 24; do
  for v in v3 gs ss v2; do
    if [ $v = v3 ]; then unset SPLINTER_HIP_LIB; else export SPLINTER_HIP_LIB=$L/libsplinter_hip_$v.so; fi
    timeout -k 10 60 $T --store hbm:$v$rep$th --threads $th --seconds 2 --keys 65536 --value-len 150 | sed "s/^{/{\"ring\": \"$v\", /" >> $O/ab.jsonl 2>> $O/ab.err || exit 1
  done
done; done
echo done
