#!/bin/bash
# Round 4 call D: full GPU suite on the parallel byte-RLE kernel, then its
# per-stream timing and the C5 / C4 file benches.
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
run t_byte 300 python -u -m pytest tests/test_gpu_byterle_columns.py -m gpu -x -q --timeout 120 --timeout-method thread || exit 1
run ab_present 300 python scripts/ab_streams.py --workload c5 --rows 2600000 --factors 1,4 --kinds PRESENT
run t_all 1000 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread || exit 1
run bf_c5 400 python scripts/bench_file.py --workload c5 --no-cpu-baseline
run bf_c4 400 python scripts/bench_file.py --workload c4 --no-cpu-baseline
echo done >> $OUT/status.log
