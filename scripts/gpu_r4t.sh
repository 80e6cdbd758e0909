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
run t_rd 900 python -u -m pytest tests/test_gpu_reader.py tests/test_gpu_workloads.py tests/test_gpu_row_reader.py tests/test_gpu_stream_order.py tests/test_gpu_hive11_overflow.py tests/test_cxx_adapter.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 200 --timeout-method thread || exit 1
run bf_c4 300 python scripts/bench_file.py --workload c4 --no-cpu-baseline --check all
run bf_c5 300 python scripts/bench_file.py --workload c5 --row-reader --no-cpu-baseline --check all
run tr_c4 300 rocprofv3 --kernel-trace --stats -d "$PWD/$OUT/tr_c4" -o run --output-format csv -- python3 scripts/bench_file.py --workload c4 --iters 1 --steady 0 --no-cpu-baseline --check none
run tr_c5 300 rocprofv3 --kernel-trace --stats -d "$PWD/$OUT/tr_c5" -o run --output-format csv -- python3 scripts/bench_file.py --workload c5 --iters 1 --steady 0 --no-cpu-baseline --check none
echo done >> $OUT/status.log
