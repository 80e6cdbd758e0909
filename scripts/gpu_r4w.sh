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
run t_k 600 python -u -m pytest tests/test_gpu_dense.py tests/test_gpu_rlev2.py -m gpu -x -q --timeout 200 --timeout-method thread || exit 1
run ph_c4 200 env ORCG_LIB=liborcgpu_prof.so python scripts/ab_streams.py --workload c4 --rows 1860000 --factors 1 --phases --kinds DATA --variants 0
run bf_c4 300 python scripts/bench_file.py --workload c4 --no-cpu-baseline --check first

run bf_c4_v6 300 python scripts/bench_file.py --workload c4 --no-cpu-baseline --check first --variant 6

run bf_c5 300 python scripts/bench_file.py --workload c5 --no-cpu-baseline --check first

for spec in repeat:12 repeat:64 shortdirect:16 shortmix:32; do
  run sw_${spec/:/_} 200 python scripts/ab_rlev2.py --data ${spec%%:*} --bits ${spec##*:} --variants 0,6 --rounds 3 --refs copy || exit 1
done
echo done >> $OUT/status.log
