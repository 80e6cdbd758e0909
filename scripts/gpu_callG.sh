#!/bin/bash
# A/B of the scan-chain dense discovery (variants 34 = union + scan, 35 =
# dense 8.5 KB + scan): parity on the dense tests through the A/B build,
# then the short-run sweep rows. Each GPU step has its own limit.
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
  return $rc
}
export TMPDIR=/tmp
run dense_ab 600 env ORCG_LIB=liborcgpu_ab.so ORCG_TEST_EXTRA_VARIANTS=34,35 python -u -m pytest tests/test_gpu_dense.py -m gpu -q -rf -x --timeout 120 --timeout-method thread || { echo "parity failed, no timing" >> $OUT/status.log; exit 0; }
for spec in ${SW_SPECS:-"repeat:12" "repeat:40" "repeat:64" "shortdirect:16" "shortmix:32" "delta:12" "random:8"}; do
  run sw_${spec/:/_} 200 python scripts/ab_rlev2.py --data ${spec%%:*} --bits ${spec##*:} --variants ${SW_VARIANTS:-0,6,34,4,35} --rounds 3 --refs copy
done
run bf_c5 400 python scripts/bench_file.py --workload c5 --cpu-threads 1
for spec in ${PH_SPECS:-"repeat:12" "shortdirect:16"}; do
  run ph_${spec/:/_} 200 env ORCG_LIB=liborcgpu_prof.so python scripts/phase_prof.py --data ${spec%%:*} --bits ${spec##*:} --variants ${PH_VARIANTS:-6,34}
done
i=0
for grp in "SQ_WAVES,SQ_INSTS_VALU,SQ_INSTS_SALU,SQ_INSTS_LDS,SQ_INSTS_VMEM_WR,SQ_INSTS_BRANCH,SQ_WAVE_CYCLES,SQ_BUSY_CYCLES" \
           "SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_VALU,SQ_ACTIVE_INST_SALU,SQ_ACTIVE_INST_LDS,SQ_WAIT_ANY,SQ_LDS_BANK_CONFLICT,SQ_ACTIVE_INST_ANY,SQ_INSTS_SMEM"; do
  i=$((i+1))
  run sqpmc_$i 120 rocprofv3 --kernel-trace --pmc ${grp//,/ } -d "$PWD/$OUT/sqpmc_$i" -o run --output-format csv -- python3 scripts/ab_rlev2.py --data repeat --bits 12 --variants 6,34 --rounds 1 --iters 3 --refs ""
done
echo done >> $OUT/status.log
