#!/bin/bash
# A/B of the two-pass expansion instances (ORCG_X_CFG) on C4 / C5 kernel stats
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
for c in ${XCFGS:-0 1 2 3}; do
  ORCG_X_CFG=$c timeout -k 10 300 python -u -m pytest tests/test_gpu_dense.py -m gpu -x -q --timeout 300 --timeout-method thread -k "two_pass or value_parallel or dense_streams" > $OUT/xt_$c.log 2>&1 || { echo "test cfg $c rc=$?" >> $OUT/status.log; exit 1; }
  for w in c4 c5; do
    ORCG_X_CFG=$c timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$PWD/$OUT/x_${w}_$c" -o run --output-format csv -- python3 scripts/bench_file.py --workload $w --iters 1 --no-cpu-baseline --check none > $OUT/x_${w}_$c.log 2>&1 || { echo "prof $w cfg $c rc=$?" >> $OUT/status.log; exit 1; }
  done
  echo "cfg $c done" >> $OUT/status.log
done
