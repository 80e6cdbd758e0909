#!/bin/bash
# round-4 measurement pass: bench line + rocprof / PMC of bench.py, file
# workloads (pyarrow legs, row reader), their kernel stats, the RLEv2 sweep
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
run bench 400 python bench.py || exit 1
run prof 300 rocprofv3 --kernel-trace --stats -d "$PWD/$OUT/prof" -o run --output-format csv -- python3 bench.py --steps 50 --warmup 100 --no-cpu-baseline --no-verify --copy-inclusive 0
run pmc_fetch 200 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d "$PWD/$OUT/pmc_fetch" -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-verify --copy-inclusive 0
run pmc_write 200 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d "$PWD/$OUT/pmc_write" -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-verify --copy-inclusive 0
run bf_c5 400 python scripts/bench_file.py --workload c5 --row-reader --cpu-threads 16
run bf_c4 400 python scripts/bench_file.py --workload c4 --row-reader --cpu-threads 16
run bf_c1 300 python scripts/bench_file.py --workload c1 --row-reader --cpu-threads 16
run tr_c5 300 rocprofv3 --kernel-trace --stats -d "$PWD/$OUT/tr_c5" -o run --output-format csv -- python3 scripts/bench_file.py --workload c5 --iters 1 --steady 0 --no-cpu-baseline --check none
run tr_c4 300 rocprofv3 --kernel-trace --stats -d "$PWD/$OUT/tr_c4" -o run --output-format csv -- python3 scripts/bench_file.py --workload c4 --iters 1 --steady 0 --no-cpu-baseline --check none
for spec in random:64 random:13 random:8 random:1 delta:12 patched:12 repeat:12 repeat:40 repeat:64 shortdirect:16 shortdirect:64 shortmix:32; do
  run sw_${spec/:/_} 200 python scripts/ab_rlev2.py --data ${spec%%:*} --bits ${spec##*:} --variants 0,2,3,6 --rounds 3 --refs copy || exit 1
done
echo done >> $OUT/status.log
