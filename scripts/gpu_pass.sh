#!/bin/bash
# One GPU-box pass: named steps, each under its own time limit; a fault,
# abort, segfault or timeout stops the pass (no further GPU work in the call).
#   scripts/gpu_pass.sh "name:seconds:command" ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
: > $OUT/status.log
export TMPDIR=/tmp
for spec in "$@"; do
  name=${spec%%:*}; rest=${spec#*:}; t=${rest%%:*}; cmd=${rest#*:}
  echo "[$(date +%T)] start $name" >> $OUT/status.log
  timeout -k 10 "$t" bash -c "$cmd" > "$OUT/$name.log" 2>&1
  rc=$?
  echo "[$(date +%T)] $name rc=$rc" >> $OUT/status.log
  case $rc in 124|137|134|139) echo "fatal rc=$rc in $name, stopping" >> $OUT/status.log; exit $rc;; esac
done
echo done >> $OUT/status.log
