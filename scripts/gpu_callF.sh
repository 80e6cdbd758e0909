#!/bin/bash
# Round-3 check after the C++ adapter fix: GPU tests, smoke, the file-path
# benches with the steady-state device decode, the dense-path phase profile
# and SQ counters of the union instance on SHORT_REPEAT 12-bit.
# Each GPU step has its own limit; a fatal status stops the script.
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
  return 0
}
export TMPDIR=/tmp
if [ -z "${SKIP_TESTS:-}" ]; then
  run pytest_gpu 900 python -u -m pytest tests -m gpu -q -rf --timeout 120 --timeout-method thread
  run smoke 120 python __graft_entry__.py smoke
fi
for w in ${BF_WORKLOADS:-c5 c4 c3}; do
  run bf_$w 600 python scripts/bench_file.py --workload $w --row-reader
done
for spec in ${PH_SPECS:-"repeat:12" "shortdirect:16"}; do
  run ph_${spec/:/_} 200 env ORCG_LIB=liborcgpu_prof.so python scripts/phase_prof.py --data ${spec%%:*} --bits ${spec##*:} --variants ${PH_VARIANTS:-6,4}
done
i=0
for grp in "SQ_WAVES,SQ_INSTS_VALU,SQ_INSTS_SALU,SQ_INSTS_LDS,SQ_INSTS_VMEM_WR,SQ_INSTS_BRANCH,SQ_WAVE_CYCLES,SQ_BUSY_CYCLES" \
           "SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_VALU,SQ_ACTIVE_INST_SALU,SQ_ACTIVE_INST_LDS,SQ_WAIT_ANY,SQ_LDS_BANK_CONFLICT,SQ_ACTIVE_INST_ANY,SQ_INSTS_SMEM"; do
  i=$((i+1))
  run sqpmc_$i 120 rocprofv3 --kernel-trace --pmc ${grp//,/ } -d "$PWD/$OUT/sqpmc_$i" -o run --output-format csv -- python3 scripts/ab_rlev2.py --data repeat --bits 12 --variants 6 --rounds 1 --iters 3 --refs ""
done
echo done >> $OUT/status.log
