#!/bin/bash
# Round 4, first call: kernel traces of the shipped file path (C5, C4) to
# find where device time goes per stripe.
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
run bf_c5 400 python scripts/bench_file.py --workload c5 --cpu-threads 16 || exit 1
run tr_c5 300 rocprofv3 --kernel-trace --stats -d "$PWD/$OUT/tr_c5" -o run --output-format csv -- python3 scripts/bench_file.py --workload c5 --iters 1 --steady 0 --no-cpu-baseline || exit 1
run bf_c4 400 python scripts/bench_file.py --workload c4 --cpu-threads 16 || exit 1
run tr_c4 300 rocprofv3 --kernel-trace --stats -d "$PWD/$OUT/tr_c4" -o run --output-format csv -- python3 scripts/bench_file.py --workload c4 --iters 1 --steady 0 --no-cpu-baseline || exit 1
echo done >> $OUT/status.log
