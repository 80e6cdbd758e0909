#!/bin/bash
# round-4 pass J: the whole GPU suite and smoke on the committed final tree
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
: > $OUT/status.log
run() {
  local name=$1 t=$2; shift 2
  echo "[$(date +%T)] start $name" >> $OUT/status.log
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "[$(date +%T)] $name rc=$rc" >> $OUT/status.log
  case $rc in 124|137|134|139) echo "fatal rc=$rc in $name, stopping" >> $OUT/status.log; exit $rc;; esac
  return $rc
}
export TMPDIR=/tmp
run j_all 800 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread || exit 1
run j_smoke 120 python __graft_entry__.py smoke || exit 1
echo done >> $OUT/status.log
