#!/bin/bash
# SQ counter passes (instruction mix, wait/active cycles, LDS) for bench.py;
# one rocprofv3 --pmc run per group, kernel-trace/stats not combined.
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
TAG=${TAG:-sq}
ARGS=${BENCH_ARGS:---steps 1 --warmup 0 --no-cpu}
OUT=$ROOT/gpurun_out/pmc_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp || exit 1
G1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH"
G2="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS"
G3="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS_LOAD SQ_INSTS_LDS_STORE SQ_IFETCH SQ_LDS_ADDR_CONFLICT SQ_BUSY_CYCLES SQ_INSTS_VALU_INT32"
i=0
for G in "$G1" "$G2" "$G3"; do
  i=$((i+1))
  # ALLOW_FAIL=1: a bench that exits 1 (a timing build that fails parity) still profiles
  timeout -k 10 ${PROF_TIMEOUT:-300} rocprofv3 --pmc $G --output-format csv -d $OUT/g$i -o pmc -- python3 $ROOT/bench.py $ARGS > $OUT/g$i.log 2>&1
  rc=$?
  if [ $rc -ne 0 ] && ! { [ -n "$ALLOW_FAIL" ] && [ $rc -eq 1 ]; }; then echo "group $i failed"; tail -20 $OUT/g$i.log; exit 1; fi
done
find $OUT -name "*counter_collection.csv"
