#!/bin/bash
# round-4 final pass B: file workloads (pyarrow legs, row reader), kernel stats, RLEv2 sweep
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
run bf_c5 400 python scripts/bench_file.py --workload c5 --row-reader --cpu-threads 16
run bf_c4 400 python scripts/bench_file.py --workload c4 --row-reader --cpu-threads 16
run bf_c1 300 python scripts/bench_file.py --workload c1 --row-reader --cpu-threads 16
run tr_c5 300 rocprofv3 --kernel-trace --stats -d "$PWD/$OUT/tr_c5" -o run --output-format csv -- python3 scripts/bench_file.py --workload c5 --iters 1 --steady 0 --no-cpu-baseline --check none
run tr_c4 300 rocprofv3 --kernel-trace --stats -d "$PWD/$OUT/tr_c4" -o run --output-format csv -- python3 scripts/bench_file.py --workload c4 --iters 1 --steady 0 --no-cpu-baseline --check none
run wl_c5 300 python bench.py --workload c5 --steps 5 --warmup 2
run ph_c4 200 env ORCG_LIB=liborcgpu_prof.so python scripts/ab_streams.py --workload c4 --rows 1860000 --factors 1 --phases --kinds DATA --variants 0
run ph_c5 200 env ORCG_LIB=liborcgpu_prof.so python scripts/ab_streams.py --workload c5 --rows 2600000 --factors 1 --phases --kinds PRESENT,DATA,LENGTH --variants 0
for spec in random:64 random:13 random:8 random:1 delta:12 patched:12 repeat:12 repeat:40 repeat:64 shortdirect:16 shortdirect:64 shortmix:32; do
  run sw_${spec/:/_} 200 python scripts/ab_rlev2.py --data ${spec%%:*} --bits ${spec##*:} --variants 0,2,3,6 --rounds 3 --refs copy || exit 1
done
echo done >> $OUT/status.log
