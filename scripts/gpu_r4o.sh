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
run t_byte 400 python -u -m pytest tests/test_gpu_byterle_columns.py tests/test_gpu_java_tree.py tests/test_gpu_reader.py tests/test_gpu_rlev1.py tests/test_gpu_row_reader.py -m gpu -x -q --timeout 200 --timeout-method thread || exit 1
run ph_pres 200 env ORCG_LIB=liborcgpu_prof.so python scripts/ab_streams.py --workload c5 --rows 2600000 --factors 1 --phases --kinds PRESENT
run bf_c5 500 python scripts/bench_file.py --workload c5 --row-reader --no-cpu-baseline --check all
run tr_c5 300 rocprofv3 --kernel-trace --stats -d "$PWD/$OUT/tr_c5" -o run --output-format csv -- python3 scripts/bench_file.py --workload c5 --iters 1 --steady 0 --no-cpu-baseline --check none
echo done >> $OUT/status.log
