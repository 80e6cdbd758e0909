#!/bin/bash
# round-4 pass I: ReaderMetrics (new C ABI) and the reader tests on the final tree, smoke
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
run i_tests 400 python -u -m pytest tests/test_gpu_reader.py tests/test_gpu_row_reader.py tests/test_cxx_adapter.py -m gpu -x -q --timeout 120 --timeout-method thread || exit 1
run i_smoke 120 python __graft_entry__.py smoke || exit 1
echo done >> $OUT/status.log
