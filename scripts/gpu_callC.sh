#!/bin/bash
# Full check + measurement call: GPU tests, smoke, bench (default and the
# driver's settings), kernel trace + PMC of the bench, RLEv2 routing sweep.
# Each GPU step has its own limit; a fatal status stops the script.
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
  return 0
}
export TMPDIR=/tmp
if [ -z "${SKIP_TESTS:-}" ]; then
  run pytest_gpu 900 python -u -m pytest tests -m gpu -q -rf -x --timeout 120 --timeout-method thread
  run smoke 120 python __graft_entry__.py smoke
fi
run bench 300 python bench.py
run bench5_a 120 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --copy-inclusive 0
run bench5_b 120 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --copy-inclusive 0
run prof 300 rocprofv3 --kernel-trace --stats -d "$PWD/$OUT/prof" -o run --output-format csv -- python3 bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-verify --copy-inclusive 0
run pmc_fetch 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d "$PWD/$OUT/pmc_fetch" -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --settle-ms 0 --no-cpu-baseline --no-verify --copy-inclusive 0
run pmc_write 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d "$PWD/$OUT/pmc_write" -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --settle-ms 0 --no-cpu-baseline --no-verify --copy-inclusive 0
for spec in ${SW_SPECS:-"random:64" "random:8" "delta:12" "patched:12" "random:13" "random:1" "repeat:12" "repeat:40" "repeat:64" "shortdirect:16" "shortdirect:64" "shortmix:32"}; do
  run sw_${spec/:/_} 200 python scripts/ab_rlev2.py --data ${spec%%:*} --bits ${spec##*:} --variants ${SW_VARIANTS:-0,2,3,4,6,7,16} --rounds 3 --refs copy,probe5
done
echo done >> $OUT/status.log
