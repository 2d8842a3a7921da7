# round 2, call 30: cross-process attach time vs hbm arena size (dmabuf IPC import)
set -x
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for n in 65536 262144 1048576; do timeout -k 10 200 python -u scripts/cli_search_debug.py $n 2>&1 | head -3 || true; done
