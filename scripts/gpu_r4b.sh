#!/bin/bash
# Round 4 call B: row-reader race/variant tests, per-stream timing at
# several segment counts (C5, C4 stripe 0).
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
run rr_tests 600 python -u -m pytest tests/test_gpu_row_reader.py tests/test_gpu_hive11_overflow.py -m gpu -x -q --timeout 120 --timeout-method thread
run ab_c5 400 python scripts/ab_streams.py --workload c5 --rows 2600000 --factors 1,4,16 --variants ${VARS:-0,6,3}
run ab_c4 400 python scripts/ab_streams.py --workload c4 --rows 1860000 --factors 1,4,16 --variants ${VARS:-0,6,3}
echo done >> $OUT/status.log
