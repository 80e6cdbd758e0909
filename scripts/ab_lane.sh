#!/bin/bash
# A/B of a reader change on configs[4]: the tree's library (liborcgpu.so)
# against liborcgpu_base.so (a copy of the build before the change),
# interleaved on one box, after the reader GPU tests on the new library.
# Used for the spare-lane, values-first and fine-stream instance A/Bs
# (profiles/r06/inv/ab_*_c5.jsonl).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
: > $OUT/status.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_reader.py tests/test_gpu_workloads.py tests/test_gpu_row_reader.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/tests.log 2>&1
rc=$?; echo "tests rc=$rc" >> $OUT/status.log; [ $rc -eq 0 ] || exit 1
for rep in 1 2 3; do
  for lib in liborcgpu_base.so liborcgpu.so; do
    timeout -k 10 150 env ORCG_LIB=$lib python scripts/bench_file.py --workload c5 --iters 3 --no-cpu-baseline --check none > $OUT/lane_${lib%.so}_$rep.log 2>&1
    rc=$?; echo "$lib $rep rc=$rc" >> $OUT/status.log
    case $rc in 124|137|134|139) exit $rc;; esac
  done
done
timeout -k 10 150 python scripts/bench_file.py --workload c5 --iters 3 --no-cpu-baseline > $OUT/lane_check.log 2>&1
echo "check rc=$?" >> $OUT/status.log
echo done >> $OUT/status.log
