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
run jobs_c4 300 env ORCG_DEBUG_JOBS=1 python scripts/bench_file.py --workload c4 --iters 1 --steady 0 --no-cpu-baseline --check none
run bf_c4_f0 300 env ORCG_FINE_PLANS=0 python scripts/bench_file.py --workload c4 --no-cpu-baseline --check first
run bf_c4_f1 300 python scripts/bench_file.py --workload c4 --no-cpu-baseline --check first
run bf_c5_f0 300 env ORCG_FINE_PLANS=0 python scripts/bench_file.py --workload c5 --no-cpu-baseline --check first
run bf_c5_f1 300 python scripts/bench_file.py --workload c5 --no-cpu-baseline --check first
run ph_c4 200 env ORCG_LIB=liborcgpu_prof.so python scripts/ab_streams.py --workload c4 --rows 1860000 --factors 1 --phases --kinds DATA,LENGTH,SECONDARY --variants 0,3,6
echo done >> $OUT/status.log
