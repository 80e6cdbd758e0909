#!/bin/bash
# Round-6 investigation pass: isolated C5 PRESENT decodes, a C5 kernel trace
# at HEAD, and the stream-shape sweep (default / two-pass / one-pass union).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
: > $OUT/status.log
step() {  # name seconds command...
  local name=$1 t=$2; shift 2
  echo "[$(date +%T)] start $name" >> $OUT/status.log
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "[$(date +%T)] $name rc=$rc" >> $OUT/status.log
  case $rc in 124|137|134|139) exit $rc;; esac
  return 0
}
for s in ${INV:-ab_present prof_c5 sweep}; do
  case $s in
    ab_present) step ab_present 200 python scripts/ab_streams.py --workload c5 --kinds PRESENT --factors 1,4,16 ;;
    prof_c5) step prof_c5 300 rocprofv3 --kernel-trace --stats -d "$PWD/$OUT/prof_c5" -o run --output-format csv -- python3 scripts/bench_file.py --workload c5 --iters 1 --no-cpu-baseline --check none ;;
    sweep) SW_VARIANTS=${SW_VARIANTS:-0,6,8} bash scripts/sweep_r06.sh; [ $? -eq 0 ] || exit 1 ;;
  esac
done
echo done >> $OUT/status.log
