#!/bin/bash
# round-4 pass G: small streams on host plans (ORCG_SMALL_STREAM) -- the whole
# GPU suite, smoke, configs[0] single / concurrent readers, C5 / C4 regression
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
run t_reader 300 python -u -m pytest tests/test_gpu_reader.py tests/test_gpu_workloads.py -m gpu -x -q --timeout 120 --timeout-method thread || exit 1
run g_c1 200 python scripts/bench_file.py --workload c1 --row-reader --cpu-threads 1,16 || exit 1
run g_c1_s0 120 env ORCG_SMALL_STREAM=0 python scripts/bench_file.py --workload c1 --iters 3 --no-cpu-baseline --check none || exit 1
run g_c1_r8 120 env GPU_MAX_HW_QUEUES=8 ORCG_LANES=1 python scripts/bench_file.py --workload c1 --readers 8 --iters 3 --no-cpu-baseline --check none --steady 0 || exit 1
run g_c1_r16 120 env GPU_MAX_HW_QUEUES=16 ORCG_LANES=1 python scripts/bench_file.py --workload c1 --readers 16 --iters 3 --no-cpu-baseline --check none --steady 0 || exit 1
run g_c5 200 python scripts/bench_file.py --workload c5 --no-cpu-baseline --check all || exit 1
run g_c4 200 python scripts/bench_file.py --workload c4 --no-cpu-baseline --check all || exit 1
run t_all 800 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread || exit 1
run smoke 120 python __graft_entry__.py smoke || exit 1
echo done >> $OUT/status.log
