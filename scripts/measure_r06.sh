#!/bin/bash
# Round-6 evidence pass: file benches (with the row reader and CPU legs) and
# rocprof kernel stats of configs[0] / [3] / [4], then the headline bench.
#   MEAS="bf_c4 bf_c5 ..." selects steps
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
step() {  # name seconds command...
  local name=$1 t=$2; shift 2
  echo "[$(date +%T)] start $name" >> $OUT/status.log
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "[$(date +%T)] $name rc=$rc" >> $OUT/status.log
  case $rc in 124|137|134|139) exit $rc;; esac
  return 0
}
for s in ${MEAS:-bf_c1 bf_c4 bf_c5 prof_c1 prof_c4 prof_c5}; do
  case $s in
    bf_c1) step bf_c1 400 python scripts/bench_file.py --workload c1 --row-reader ;;
    bf_c3) step bf_c3 600 python scripts/bench_file.py --workload c3 --row-reader ;;
    bf_c4) step bf_c4 400 python scripts/bench_file.py --workload c4 --row-reader ;;
    bf_c5) step bf_c5 400 python scripts/bench_file.py --workload c5 --row-reader ;;
    prof_c1|prof_c4|prof_c5)
      w=${s#prof_}
      step $s 400 rocprofv3 --kernel-trace --stats -d "$PWD/$OUT/$s" -o run --output-format csv -- python3 scripts/bench_file.py --workload $w --iters 1 --no-cpu-baseline --check none ;;
    bench) step bench 400 python bench.py ;;
    prof_c2) step prof_c2 400 rocprofv3 --kernel-trace --stats -d "$PWD/$OUT/prof_c2" -o run --output-format csv -- python3 bench.py --steps 50 --warmup 100 --no-cpu-baseline --no-verify --copy-inclusive 0 ;;
    pmc_fetch|pmc_write)
      c=FETCH_SIZE; [ $s = pmc_write ] && c=WRITE_SIZE
      step $s 300 timeout -s KILL 280 rocprofv3 --kernel-trace --pmc $c -d "$PWD/$OUT/$s" -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-verify --copy-inclusive 0 ;;
    smoke) step smoke 300 python __graft_entry__.py smoke ;;
  esac
done
echo done >> $OUT/status.log
