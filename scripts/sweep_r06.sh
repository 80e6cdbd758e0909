#!/bin/bash
# Stream-shape sweep of the default and the pinned instances (product library)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
V=${SW_VARIANTS:-0,3,6,8}
for spec in ${SW_SPECS:-"repeat:12" "repeat:64" "shortdirect:16" "shortdirect:64" "shortmix:32" "random:8" "delta:12" "patched:12" "random:64"}; do
  timeout -k 10 300 env ORCG_LIB=liborcgpu.so python scripts/ab_rlev2.py --data ${spec%%:*} --bits ${spec##*:} --variants $V --rounds 3 --refs copy > $OUT/sw_${spec/:/_}.log 2>&1
  rc=$?; echo "sweep $spec rc=$rc" >> $OUT/status.log
  case $rc in 124|137|134|139) exit $rc;; esac
done
