#!/bin/bash
# round-4 pass F: configs[0] with concurrent readers, with and without side
# lanes (ORCG_LANES=1: one stream per reader; HIP maps streams onto 4 hardware queues)
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
for k in 2 4 8; do
  run c1_r${k} 120 python scripts/bench_file.py --workload c1 --readers $k --iters 3 --no-cpu-baseline --check none --steady 0 || exit 1
  run c1_r${k}_l1 120 env ORCG_LANES=1 python scripts/bench_file.py --workload c1 --readers $k --iters 3 --no-cpu-baseline --check none --steady 0 || exit 1
done
run c1_r4_hw8 120 env GPU_MAX_HW_QUEUES=8 python scripts/bench_file.py --workload c1 --readers 4 --iters 3 --no-cpu-baseline --check none --steady 0 || exit 1
run c1_r8_hw8_l1 120 env GPU_MAX_HW_QUEUES=8 ORCG_LANES=1 python scripts/bench_file.py --workload c1 --readers 8 --iters 3 --no-cpu-baseline --check none --steady 0 || exit 1
echo done >> $OUT/status.log
