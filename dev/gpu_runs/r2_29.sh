# round 2, call 29: CLI verbs against an hbm: store owned by another process (debug)
set -x
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 200 python -u scripts/cli_search_debug.py 4096 &&
timeout -k 10 200 python -u scripts/cli_search_debug.py 2097152
