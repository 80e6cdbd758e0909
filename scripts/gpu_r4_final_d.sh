#!/bin/bash
# round-4 pass D: the whole GPU suite on the final tree, smoke, configs[0]
# (demo-11, 385 small stripes) with concurrent readers, C5 regression check
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
run t_reader 300 python -u -m pytest tests/test_gpu_reader.py -m gpu -x -q --timeout 120 --timeout-method thread || exit 1
run t_all 800 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread || exit 1
run smoke 120 python __graft_entry__.py smoke || exit 1
run bf_c1 300 python scripts/bench_file.py --workload c1 --row-reader --readers 4 --cpu-threads 1,16 || exit 1
run bf_c1_r8 200 python scripts/bench_file.py --workload c1 --readers 8 --no-cpu-baseline --check none --steady 0 || exit 1
run bf_c1_r16 200 python scripts/bench_file.py --workload c1 --readers 16 --no-cpu-baseline --check none --steady 0 || exit 1
run bf_c5 300 python scripts/bench_file.py --workload c5 --no-cpu-baseline --check first || exit 1
echo done >> $OUT/status.log
