#!/bin/bash
# Round-6 final evidence at HEAD, in two calls (FINAL=b / c):
#  b: RLEv2 GPU tests, the short DIRECT 64-bit / DIRECT 64-bit sweep rows,
#     the headline bench, C4 / C5 file benches (row reader) + kernel stats
#  c: C1 / C3 file benches (row reader) + C1 kernel stats
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
: > $OUT/status.log
if [ "${FINAL:-b}" = b ]; then
  timeout -k 10 500 python -u -m pytest tests/test_gpu_dense.py tests/test_gpu_rlev2.py tests/test_gpu_fullsize.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/tests_rlev2.log 2>&1
  rc=$?; echo "tests_rlev2 rc=$rc" >> $OUT/status.log; [ $rc -eq 0 ] || exit 1
  SW_VARIANTS=0,6 SW_SPECS="shortdirect:64 random:64" bash scripts/sweep_r06.sh || exit 1
  MEAS="bench bf_c4 bf_c5 prof_c4 prof_c5" bash scripts/measure_r06.sh
else
  MEAS="bf_c1 prof_c1 bf_c3" bash scripts/measure_r06.sh
fi
