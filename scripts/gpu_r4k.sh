#!/bin/bash
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
run t_all 800 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread || exit 1
run bf_c5 500 python scripts/bench_file.py --workload c5 --row-reader --cpu-threads 1,16
run tr_c5 300 rocprofv3 --kernel-trace --stats -d "$PWD/$OUT/tr_c5" -o run --output-format csv -- python3 scripts/bench_file.py --workload c5 --iters 1 --steady 0 --no-cpu-baseline --check none
run bf_c4 400 python scripts/bench_file.py --workload c4 --row-reader --cpu-threads 1,16
run ph_c5 200 env ORCG_LIB=liborcgpu_prof.so python scripts/ab_streams.py --workload c5 --rows 2600000 --factors 1 --phases --kinds DATA,LENGTH --variants 0,2,6
run ph_c4 200 env ORCG_LIB=liborcgpu_prof.so python scripts/ab_streams.py --workload c4 --rows 1860000 --factors 1 --phases --kinds DATA,LENGTH --variants 0,2,6
run bf_c1 300 python scripts/bench_file.py --workload c1 --row-reader --cpu-threads 1,16
echo done >> $OUT/status.log
