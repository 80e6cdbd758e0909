#!/bin/bash
# One GPU-box session: each GPU step has its own time limit; a fault, abort,
# segfault or timeout stops the session (no further GPU work in this call).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p $OUT
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
STEPS="${*:-pytest smoke bench prof}"
for s in $STEPS; do
  case $s in
    info) run info 60 bash -c "rocm-smi --showproductname; nproc; lscpu | grep 'Model name'" ;;
    pytest) run pytest_gpu 1200 python -u -m pytest tests -m gpu -q -rf -x --timeout 120 --timeout-method thread ;;
    pytestcpu) run pytest_cpu 600 python -m pytest tests -m "not gpu" -q ;;
    smoke) run smoke 300 python __graft_entry__.py smoke ;;
    bench) run bench 600 python bench.py ;;
    drift) run drift 300 python scripts/drift.py ;;
    ab) run ab 600 python scripts/ab_rlev2.py --variants 0,1,8,9 ;;
    ab13) run ab13 600 python scripts/ab_rlev2.py --bits 13 --variants 0,1,8,9 ;;
    sweep)
      for b in 1 8 13 24 32 48 64; do run sweep_w$b 300 python scripts/ab_rlev2.py --bits $b --variants 0,1,8,9,10,11,14,15,16,18,19 --rounds 3 || true; done
      for d in delta repeat patched; do run sweep_$d 300 python scripts/ab_rlev2.py --data $d --bits 12 --variants 0,1,8,9,10,11,14,15,16,18,19 --rounds 3 || true; done
      run sweep_repeat40 300 python scripts/ab_rlev2.py --data repeat --bits 40 --variants 0,1,8,9,10,11,14,15,16,18,19 --rounds 3 || true ;;
    cliff)
      # short-run shapes at >= 1.25 B/value (the density rule's serial instances) and wide SHORT_REPEAT
      V=${CLIFF_VARIANTS:-0,8,10,11,15,16,19,20}
      run cliff_repeat64 300 python scripts/ab_rlev2.py --data repeat --bits 64 --variants $V --rounds 3 --refs probe5 || true
      run cliff_repeat40 300 python scripts/ab_rlev2.py --data repeat --bits 40 --variants $V --rounds 3 --refs probe5 || true
      run cliff_repeat12 300 python scripts/ab_rlev2.py --data repeat --bits 12 --variants $V --rounds 3 --refs probe5 || true
      run cliff_sdir16 300 python scripts/ab_rlev2.py --data shortdirect --bits 16 --variants $V --rounds 3 --refs probe5 || true
      run cliff_sdir64 300 python scripts/ab_rlev2.py --data shortdirect --bits 64 --variants $V --rounds 3 --refs probe5 || true
      run cliff_smix32 300 python scripts/ab_rlev2.py --data shortmix --bits 32 --variants $V --rounds 3 --refs probe5 || true ;;
    dense2)
      V=${D2_VARIANTS:-19,21,22,23,24}
      for spec in "repeat 12" "repeat 40" "repeat 64" "shortdirect 16" "shortdirect 64" "shortmix 32" "random 8" "delta 12" "random 64"; do
        set -- $spec
        run d2_$1_$2 300 python scripts/ab_rlev2.py --data $1 --bits $2 --variants $V --rounds 3 --refs copy || true
      done ;;
    phase)
      V=${PH_VARIANTS:-19,21}
      for spec in ${PH_SPECS:-"repeat:12" "shortdirect:16" "repeat:64"}; do
        run ph_${spec/:/_} 300 env ORCG_LIB=liborcgpu_prof.so python scripts/phase_prof.py --data ${spec%%:*} --bits ${spec##*:} --variants $V || true
      done ;;
    sqpmc)
      # SQ counters of one instance on one stream shape (separate passes)
      export TMPDIR=/tmp
      V=${SQ_VARIANT:-21}; D=${SQ_DATA:-repeat}; B=${SQ_BITS:-12}
      i=0
      for grp in "SQ_WAVES,SQ_INSTS_VALU,SQ_INSTS_SALU,SQ_INSTS_LDS,SQ_INSTS_VMEM_WR,SQ_INSTS_BRANCH,SQ_WAVE_CYCLES,SQ_BUSY_CYCLES" \
                 "SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_VALU,SQ_ACTIVE_INST_SALU,SQ_ACTIVE_INST_LDS,SQ_WAIT_ANY,SQ_LDS_BANK_CONFLICT,SQ_ACTIVE_INST_ANY,SQ_INSTS_SMEM"; do
        i=$((i+1))
        run sqpmc_$i 120 rocprofv3 --kernel-trace --pmc ${grp//,/ } -d "$PWD/$OUT/sqpmc_$i" -o run --output-format csv -- python3 scripts/ab_rlev2.py --data $D --bits $B --variants $V --rounds 1 --iters 3 --refs "" || break
      done ;;
    sweep2)
      V=${SW_VARIANTS:-0,2,3,4,5,16,20}
      for spec in ${SW_SPECS:-"random:64" "random:48" "random:13" "random:8" "random:1" "delta:12" "patched:12" "repeat:12" "repeat:40" "repeat:64" "shortdirect:16" "shortdirect:64" "shortmix:32"}; do
        run sw_${spec/:/_} 300 python scripts/ab_rlev2.py --data ${spec%%:*} --bits ${spec##*:} --variants $V --rounds 3 --refs copy,probe5 || true
      done ;;
    tnew) run tnew 900 python -u -m pytest tests/test_gpu_java_tree.py tests/test_gpu_row_reader.py tests/test_cxx_adapter.py tests/test_gpu_reader.py -m gpu -q -rf -x --timeout 120 --timeout-method thread ;;
    tfile) run tfile 900 python -u -m pytest ${TFILE_TESTS:-tests/test_gpu_reader.py} -m gpu -q -rf -x --timeout 120 --timeout-method thread ;;
    bench5)
      # the driver's settings (--steps 20 --warmup 5), variants interleaved
      for v in ${B5_VARIANTS:-0 7 0 7}; do run bench5_v$v 300 python bench.py --steps 20 --warmup 5 --variant $v --no-cpu-baseline --copy-inclusive 0; cat $OUT/bench5_v$v.log >> $OUT/bench5_all.log; done ;;
    ab64) run ab64 300 python scripts/ab_rlev2.py --data random --bits 64 --variants ${AB_VARIANTS:-0,2,7,20} --rounds 5 --refs copy,probe5 ;;
    bf) for w in ${BF_WORKLOADS:-c5 c4 c3}; do run bf_$w 600 python scripts/bench_file.py --workload $w --row-reader ${BF_ARGS:-}; done ;;
    proffile)
      export TMPDIR=/tmp
      for w in ${PF_WORKLOADS:-c5}; do run prof_$w 600 rocprofv3 --kernel-trace --stats -d "$PWD/$OUT/prof_$w" -o run --output-format csv -- python3 scripts/bench_file.py --workload $w --iters 1 --no-cpu-baseline; done ;;
    dbg11) run dbg11 300 python scripts/dbg_file11.py ;;
    treader) run treader 600 python -u -m pytest tests/test_gpu_reader.py -m gpu -q -rf -x --timeout 120 --timeout-method thread ;;
    benchwalk) run bench_walk 600 python bench.py --variant 1 --no-cpu-baseline ;;
    prof)
      export TMPDIR=/tmp
      run prof 600 rocprofv3 --kernel-trace --stats -d "$PWD/$OUT/prof" -o run --output-format csv -- python3 bench.py --steps 50 --warmup 100 --no-cpu-baseline --no-verify --copy-inclusive 0 ;;
    pmc)
      export TMPDIR=/tmp
      run pmc_fetch 600 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d "$PWD/$OUT/pmc_fetch" -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-verify --copy-inclusive 0
      run pmc_write 600 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d "$PWD/$OUT/pmc_write" -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-verify --copy-inclusive 0 ;;
    *) echo "unknown step $s" >> $OUT/status.log ;;
  esac
done
echo done >> $OUT/status.log
