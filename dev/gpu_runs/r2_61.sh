# round 2, call 61: host-API A/B in one box, interleaved: ring v3 (default) vs v2 (previous commit)
set -x
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r2_61
mkdir -p $O
T=libsplinter_amd/bin/splinter_hostapi_bench
L=$PWD/libsplinter_amd/lib
for rep in 1 2; do for th in 1 4 8 16 24; do
  timeout -k 10 60 $T --store hbm:x$rep$th --threads $th --seconds 2 --keys 65536 --value-len 150 | sed "s/^{/{\"ring\": \"v3\", /" >> $O/ab.jsonl 2>> $O/ab.err || exit 1
  SPLINTER_HIP_LIB=$L/libsplinter_hip_v2.so timeout -k 10 60 $T --store hbm:y$rep$th --threads $th --seconds 2 --keys 65536 --value-len 150 | sed "s/^{/{\"ring\": \"v2\", /" >> $O/ab.jsonl 2>> $O/ab.err || exit 1
done; done
echo done
