#!/bin/bash
# Round-3 check of the committed tree: GPU tests, smoke, the C2 bench, the
# file-path benches (C5 / C4 / C3 with the RowReader leg and the pyarrow CPU
# legs), kernel traces of the C5 / C4 decodes, and the default's sweep.
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
  run pytest_gpu 900 python -u -m pytest tests -m gpu -q -rf --timeout 120 --timeout-method thread
  run smoke 120 python __graft_entry__.py smoke
fi
run bench 300 python bench.py
for w in ${BF_WORKLOADS:-c5 c4 c3}; do
  run bf_$w 600 python scripts/bench_file.py --workload $w --row-reader
done
for w in ${PF_WORKLOADS:-c5 c4}; do
  run prof_$w 300 rocprofv3 --kernel-trace --stats -d "$PWD/$OUT/prof_$w" -o run --output-format csv -- python3 scripts/bench_file.py --workload $w --iters 1 --no-cpu-baseline
done
for spec in ${SW_SPECS:-"random:64" "random:13" "random:8" "random:1" "delta:12" "patched:12" "repeat:12" "repeat:40" "repeat:64" "shortdirect:16" "shortdirect:64" "shortmix:32"}; do
  run sw_${spec/:/_} 200 python scripts/ab_rlev2.py --data ${spec%%:*} --bits ${spec##*:} --variants ${SW_VARIANTS:-0,3,6,16} --rounds 3 --refs copy,probe5
done
run ab64 300 python scripts/ab_rlev2.py --data random --bits 64 --variants ${AB_VARIANTS:-0,2,31,32,33} --rounds 5 --refs copy,probe5
echo done >> $OUT/status.log
