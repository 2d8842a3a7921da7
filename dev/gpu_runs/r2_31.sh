# round 2, call 31: second-process attach (hipIpcOpenMemHandle, dmabuf) time vs arena size
set -x
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for n in 262144 500000 640000 1000000; do timeout -k 10 120 python -u scripts/ipc_open_debug.py $n || true; done
