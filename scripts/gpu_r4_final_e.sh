#!/bin/bash
# round-4 pass E: pinned-variant file test, then configs[3] at its per-GPU
# size (1.25 * 10^8 rows), every stripe checked against pyarrow
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
run t_variant 240 python -u -m pytest tests/test_gpu_reader.py -m gpu -x -q -k "pinned_variant or concurrent" --timeout 120 --timeout-method thread || exit 1
run bf_c4_125m 900 python -u scripts/bench_file.py --workload c4 --rows 125000000 --cpu-threads 16 --iters 2 --steady 3 --check all || exit 1
echo done >> $OUT/status.log
