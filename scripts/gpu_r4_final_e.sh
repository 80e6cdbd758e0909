#!/bin/bash
# round-4 pass E: kernel + runtime trace of the configs[0] scan (385 small
# stripes: where the per-stripe fixed cost goes), then configs[3] at its
# per-GPU size (1.25 * 10^8 rows), every stripe checked against pyarrow
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
run tr_c1 150 rocprofv3 --kernel-trace --runtime-trace --stats -d "$PWD/$OUT/tr_c1" -o run --output-format csv -- python3 scripts/bench_file.py --workload c1 --iters 1 --steady 0 --no-cpu-baseline --check none || exit 1
run bf_c4_125m 900 python -u scripts/bench_file.py --workload c4 --rows 125000000 --cpu-threads 16 --iters 1 --steady 2 --check all || exit 1
echo done >> $OUT/status.log
