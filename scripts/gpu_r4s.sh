#!/bin/bash
# round-4 RLEv2 sweep (stream shapes of profiles/r03/sweep.md)
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
for spec in ${SW_SPECS:-random:64 random:13 random:8 random:1 delta:12 patched:12 repeat:12 repeat:40 repeat:64 shortdirect:16 shortdirect:64 shortmix:32}; do
  run sw_${spec/:/_} 200 python scripts/ab_rlev2.py --data ${spec%%:*} --bits ${spec##*:} --variants ${SW_VARIANTS:-0,2,3,6} --rounds 3 --refs copy || exit 1
done
echo done >> $OUT/status.log
