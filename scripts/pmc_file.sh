#!/bin/bash
# SQ counter passes (one rocprofv3 --pmc run each) over one file-bench scan:
#   scripts/pmc_file.sh <workload> <tag>   (extra env, e.g. ORCG_ONE_PASS=1, passes through)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
W=$1; TAG=$2
export TMPDIR=/tmp
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_SMEM" \
           "SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_VMEM_WR"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $grp -d "$PWD/gpurun_out/pmc_${W}_${TAG}_$i" -o run --output-format csv -- python3 scripts/bench_file.py --workload $W --iters 1 --no-cpu-baseline --check none --steady 1 > gpurun_out/pmc_${W}_${TAG}_$i.log 2>&1 || exit $?
done
