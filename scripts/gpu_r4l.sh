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
run t_kern 600 python -u -m pytest tests/test_gpu_dense.py tests/test_gpu_rlev2.py tests/test_gpu_byterle_columns.py tests/test_gpu_reader.py tests/test_gpu_workloads.py -m gpu -x -q --timeout 200 --timeout-method thread || exit 1
run ph_c5 200 env ORCG_LIB=liborcgpu_prof.so python scripts/ab_streams.py --workload c5 --rows 2600000 --factors 1 --phases --kinds DATA,LENGTH --variants 0,2,6
run ph_c4 200 env ORCG_LIB=liborcgpu_prof.so python scripts/ab_streams.py --workload c4 --rows 1860000 --factors 1 --phases --kinds DATA,LENGTH --variants 0,2,6
run pin 120 python scripts/pinned_read.py
run bf_c5 500 python scripts/bench_file.py --workload c5 --row-reader --cpu-threads 16
run tr_c5 300 rocprofv3 --kernel-trace --stats -d "$PWD/$OUT/tr_c5" -o run --output-format csv -- python3 scripts/bench_file.py --workload c5 --iters 1 --steady 0 --no-cpu-baseline --check none
run bf_c4 400 python scripts/bench_file.py --workload c4 --cpu-threads 16
run tr_c4 300 rocprofv3 --kernel-trace --stats -d "$PWD/$OUT/tr_c4" -o run --output-format csv -- python3 scripts/bench_file.py --workload c4 --iters 1 --steady 0 --no-cpu-baseline --check none
run sw_rep 200 python scripts/ab_rlev2.py --data repeat --bits 12 --variants 0,6 --rounds 3 --refs copy
run sw_sd16 200 python scripts/ab_rlev2.py --data shortdirect --bits 16 --variants 0,6 --rounds 3 --refs copy
echo done >> $OUT/status.log
