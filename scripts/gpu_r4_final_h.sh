#!/bin/bash
# round-4 pass H (final tree, with ReaderMetrics): reader / workload GPU tests, smoke, the bench
# line, rocprof of bench.py, C1 single + 16 concurrent readers
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
run h_tests 500 python -u -m pytest tests/test_gpu_reader.py tests/test_gpu_workloads.py tests/test_gpu_row_reader.py tests/test_cxx_adapter.py tests/test_gpu_rlev2.py -m gpu -x -q --timeout 120 --timeout-method thread || exit 1
run h_smoke 120 python __graft_entry__.py smoke || exit 1
run h_bench 300 python bench.py || exit 1
run h_prof 200 rocprofv3 --kernel-trace --stats -d "$PWD/$OUT/h_prof" -o run --output-format csv -- python3 bench.py --steps 50 --warmup 100 --no-cpu-baseline --no-verify --copy-inclusive 0 || exit 1
run h_c1 120 python scripts/bench_file.py --workload c1 --iters 3 --no-cpu-baseline --check all || exit 1
run h_c1_r16 120 env GPU_MAX_HW_QUEUES=16 ORCG_LANES=1 python scripts/bench_file.py --workload c1 --readers 16 --iters 3 --no-cpu-baseline --check none --steady 0 || exit 1
echo done >> $OUT/status.log
