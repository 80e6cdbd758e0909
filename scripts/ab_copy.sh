#!/bin/bash
# The row reader's batch copies on configs[3]'s file shape (c4): helper
# count (ORCG_COPY_THREADS) x capacity, REPS runs each (SPECS="threads:capacity ...")
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
W=${W:-c4}
timeout -k 10 300 python scripts/bench_file.py --workload $W --iters 1 --no-cpu-baseline --check none > $OUT/abc_make.log 2>&1 || exit $?
F=$(ls /tmp/orcg_${W}_*.orc | head -1)
g++ -std=c++17 -O2 -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include tests/cxx/reader_test.cpp -o /tmp/rt -Lorc_amd -lorcgpu \
  -Wl,-rpath,$PWD/orc_amd -Wl,-rpath,/opt/rocm/lib || exit 1
for spec in ${SPECS:-3:1024 5:1024 3:16384}; do
  set -- ${spec//:/ }
  for rep in $(seq ${REPS:-2}); do
    r=$(ORCG_COPY_THREADS=$1 timeout -k 10 30 /tmp/rt $F --bench --batch $2 2>>$OUT/abc_err.log); rc=$?
    [ $rc = 0 ] || { echo "fail $spec rc=$rc" >> $OUT/abc.log; exit 1; }
    echo "$W thr=$1 cap=$2 rep=$rep $r" >> $OUT/abc.log
  done
done
echo done >> $OUT/abc.log
