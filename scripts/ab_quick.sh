#!/bin/bash
# Quick interleaved A/B of RLEv2 variants on several stream shapes (product
# library), plus optional file-bench debug runs. Each step has its own limit;
# a fatal status stops the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
V=${ABQ_VARIANTS:-4,6}
for spec in ${ABQ_SPECS:-"repeat:12" "repeat:64" "shortdirect:16"}; do
  timeout -k 10 200 env ORCG_LIB=liborcgpu.so python scripts/ab_rlev2.py --data ${spec%%:*} --bits ${spec##*:} --variants $V --rounds ${ABQ_ROUNDS:-3} --refs copy > $OUT/abq_${spec/:/_}.log 2>&1
  rc=$?; echo "abq $spec rc=$rc" >> $OUT/status.log
  case $rc in 124|137|134|139) exit $rc;; esac
done
if [ -n "${ABQ_FILE:-}" ]; then
  timeout -k 10 300 env ORCG_DEBUG=jobs python scripts/bench_file.py --workload $ABQ_FILE --rows ${ABQ_FILE_ROWS:-2000000} --iters 1 --no-cpu-baseline > $OUT/file_$ABQ_FILE.log 2>&1
  echo "file rc=$?" >> $OUT/status.log
fi
exit 0
