#!/bin/bash
# Debug + measurement call: decimal.orc read under pinned variants, file/RLEv2
# GPU tests, the clock-ramp probe and a short routing sweep. Each GPU step has
# its own limit; a fatal status stops the script.
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
run dbg_dec 120 env ORCG_DEBUG_ALLOC=1 ORCG_DEBUG_JOBS=1 python scripts/dbg_dec.py
run t_sub 600 python -u -m pytest tests/test_cxx_adapter.py tests/test_gpu_reader.py tests/test_gpu_rlev2.py tests/test_gpu_fullsize.py -m gpu -q -rf --timeout 120 --timeout-method thread
run ramp 200 python scripts/ramp_probe.py
for spec in ${SW_SPECS:-"random:8" "delta:12" "patched:12" "random:13" "repeat:12" "repeat:64" "shortdirect:16"}; do
  run sw_${spec/:/_} 200 python scripts/ab_rlev2.py --data ${spec%%:*} --bits ${spec##*:} --variants ${SW_VARIANTS:-0,3,4,16} --rounds 3 --refs copy
done
echo done >> $OUT/status.log
