set -x
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --list-avail > gpurun_out/pmc_list13.txt 2>&1
echo rc=$?
