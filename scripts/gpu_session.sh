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
    benchwalk) run bench_walk 600 python bench.py --variant 1 --no-cpu-baseline ;;
    prof)
      export TMPDIR=/tmp
      run prof 600 rocprofv3 --kernel-trace --stats -d "$PWD/$OUT/prof" -o run --output-format csv -- python3 bench.py --steps 50 --warmup 100 --no-cpu-baseline --no-verify --copy-inclusive 0 ;;
    pmc)
      export TMPDIR=/tmp
      run pmc_fetch 600 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d "$PWD/$OUT/pmc_fetch" -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-verify
      run pmc_write 600 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d "$PWD/$OUT/pmc_write" -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-verify ;;
    *) echo "unknown step $s" >> $OUT/status.log ;;
  esac
done
echo done >> $OUT/status.log
