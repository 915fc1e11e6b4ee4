#!/bin/bash
# round 5: Ukkonen forward sweep alone (no backtrace build) against the whole
# kernel, D_ukkonen and D_ukkonen_64k
cd "$(dirname "$0")/../.." || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/r5x
mkdir -p $OUT
for C in ${CONFIGS:-D_ukkonen_64k D_ukkonen}; do
  echo "[$(date +%T)] $C default / forward only"
  timeout -k 10 300 python bench.py --config $C --steps 3 --warmup 1 --no-cpu > $OUT/bench_$C.log 2>&1 || { tail -20 $OUT/bench_$C.log; exit 1; }
  GWAMD_DIAG=1 GWAMD_LIBRARY=claragenomicsanalysis_amd/lib/exp5/libgwamd.so timeout -k 10 300 python bench.py --config $C --steps 3 --warmup 1 --no-cpu > $OUT/bench_${C}_fwd.log 2>&1
  rc=$?; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then tail -20 $OUT/bench_${C}_fwd.log; exit 1; fi
  grep -h "kernel_only\|Error\|error" $OUT/bench_${C}_fwd.log | tail -3
done
echo "[$(date +%T)] done"
