#!/bin/bash
# round 5: where D_ukkonen_64k's time goes (forward sweep alone vs the whole
# kernel) and its SQ counters
cd "$(dirname "$0")/../.." || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/r5j
mkdir -p $OUT
for C in D_ukkonen_64k D_ukkonen D_banded_64k; do
  echo "[$(date +%T)] $C default / forward only"
  timeout -k 10 300 python bench.py --config $C --steps 2 --warmup 1 --no-cpu > $OUT/bench_$C.log 2>&1 || { tail -20 $OUT/bench_$C.log; exit 1; }
  GWAMD_DIAG=1 GWAMD_LIBRARY=claragenomicsanalysis_amd/lib/exp4/libgwamd.so timeout -k 10 300 python bench.py --config $C --steps 2 --warmup 1 --no-cpu > $OUT/bench_${C}_fwd.log 2>&1
  rc=$?; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then tail -20 $OUT/bench_${C}_fwd.log; exit 1; fi
done
echo "[$(date +%T)] sq D_ukkonen_64k"
TAG=r5j_Duk64 PROF_TIMEOUT=200 BENCH_ARGS="--config D_ukkonen_64k --steps 1 --warmup 0 --no-cpu" bash scripts/pmc_sq.sh > $OUT/sq.log 2>&1 || { tail -20 $OUT/sq.log; exit 1; }
echo "[$(date +%T)] done"
