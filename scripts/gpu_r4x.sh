#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 env ORCG_DEBUG_DEFER=1 ORCG_DEBUG_JOBS=1 python scripts/bench_file.py --workload c4 --iters 1 --steady 0 --no-cpu-baseline --check none > $OUT/defer.log 2>&1
