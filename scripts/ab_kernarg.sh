#!/bin/bash
# A/B of HIP's kernel-argument placement on the file decode (C5 / C4):
# hipLaunchKernel blocked 60-80 us per call while the GPU idled mid-stripe
# (profiles/r06/inv/hip_api_c5_548c478.txt), with the kernel starting ~2 us
# after the call returned.  KA_TESTS=1 first runs the reader GPU tests.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
: > $OUT/status.log
run() {  # name env... -- args
  local name=$1 t=$2; shift 2
  timeout -k 10 $t env "$@" > $OUT/$name.log 2>&1
  local rc=$?; echo "$name rc=$rc" >> $OUT/status.log
  case $rc in 124|137|134|139) exit $rc;; esac
  [ "$name" != tests ] || [ $rc -eq 0 ] || exit 1
}
if [ "${KA_TESTS:-0}" = 1 ]; then
  run tests 400 X=1 python -u -m pytest tests/test_gpu_reader.py tests/test_gpu_workloads.py tests/test_gpu_row_reader.py tests/test_gpu_byterle_columns.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
fi
for w in ${KA_WORK:-c5 c4}; do
  run ka_${w}_check 200 X=1 python scripts/bench_file.py --workload $w --iters 3 --no-cpu-baseline
  for rep in 1 2; do
    run ka_${w}_def_$rep 150 X=1 python scripts/bench_file.py --workload $w --iters 3 --no-cpu-baseline --check none
    run ka_${w}_host_$rep 150 HIP_FORCE_DEV_KERNARG=0 python scripts/bench_file.py --workload $w --iters 3 --no-cpu-baseline --check none
  done
done
timeout -k 10 200 rocprofv3 --kernel-trace --hip-trace --output-format csv -d "$PWD/$OUT/ht_c5" -o run -- python3 scripts/bench_file.py --workload c5 --iters 1 --no-cpu-baseline --check none > $OUT/ht_c5.log 2>&1
echo "trace rc=$?" >> $OUT/status.log
echo done >> $OUT/status.log
