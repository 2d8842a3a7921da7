#!/usr/bin/env bash
# CLI regression: every verb as a SEPARATE process against one store, checking
# exit codes (the reference's splinterctl_tests.sh contract) plus a few outputs.
# Usage: tests/cli_regression.sh [bin_dir]
set -u
BIN="${1:-$(cd "$(dirname "$0")/.." && pwd)/libsplinter_amd/bin}"
HERE="$(cd "$(dirname "$0")" && pwd)"
STORE="cli_regression_$$"
CTL="$BIN/splinterctl"
n=0; failed=0
step() {  # step "description" command...
  local what="$1"; shift
  n=$((n + 1))
  if "$@" > /tmp/cli_regression_$$.out 2>&1; then
    echo "ok $n - $what"
  else
    echo "not ok $n - $what"; sed 's/^/#   /' /tmp/cli_regression_$$.out; failed=$((failed + 1))
  fi
}
expect() {  # expect "needle" command...: command succeeds and prints needle
  local needle="$1"; shift
  "$@" | grep -qF -- "$needle"
}
step "init store"                 "$CTL" init "$STORE"
step "set a key"                  "$CTL" --use "$STORE" set test_key test_value
step "get a key"                  expect test_value "$CTL" --use "$STORE" get test_key
step "key metadata"               expect "key:        test_key" "$CTL" --use "$STORE" head test_key
step "list keys"                  expect test_key "$CTL" --use "$STORE" list
step "type a key"                 "$CTL" --use "$STORE" type test_key vartext
step "read key type"              expect SPL_SLOT_TYPE_VARTEXT "$CTL" --use "$STORE" type test_key
step "lua script"                 "$CTL" --use "$STORE" lua "$HERE/data/bus_check.lua"
step "unset a key"                "$CTL" --use "$STORE" unset test_key
step "global config"              expect "version:     4" "$CTL" --use "$STORE" config
step "set config flag"            "$CTL" --use "$STORE" config av 1
step "export json"                expect total_slots "$CTL" --use "$STORE" export
step "set bump key"               "$CTL" --use "$STORE" set bump_key "Bump Value"
step "bump the key"               "$CTL" --use "$STORE" bump bump_key
step "append to the key"          "$CTL" --use "$STORE" append bump_key "more"
step "uuid"                       "$CTL" uuid
step "label + bind"               "$CTL" --use "$STORE" bind 0x20 5
step "shard table"                "$CTL" --use "$STORE" shard table
step "stats"                      expect active_keys "$CTL" --use "$STORE" stats
step "caps"                       expect lua=yes "$CTL" caps
rm -f /tmp/cli_regression_$$.out /dev/shm/"$STORE"
echo "1..$n"
if [ "$failed" -ne 0 ]; then echo "# $failed failed"; exit 1; fi
echo "# all passed"
