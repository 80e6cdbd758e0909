#!/bin/bash
# round-4 pass C: configs[3] at its per-GPU size (1.25 * 10^8 rows), every stripe checked against pyarrow
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
: > $OUT/status.log
export TMPDIR=/tmp
echo "[$(date +%T)] start bf_c4_125m" >> $OUT/status.log
timeout -k 10 1100 python -u scripts/bench_file.py --workload c4 --rows 125000000 --cpu-threads 16 --iters 2 --steady 3 --check all > $OUT/bf_c4_125m.log 2>&1
echo "[$(date +%T)] bf_c4_125m rc=$?" >> $OUT/status.log
