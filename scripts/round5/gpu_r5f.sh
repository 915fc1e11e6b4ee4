#!/bin/bash
# round 5 timing experiment on config C's anti-diagonal pass: ring loads
# prefetched two steps ahead (exp2), and that without code stores (exp3)
cd "$(dirname "$0")/../.." || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/r5f
mkdir -p $OUT
echo "[$(date +%T)] C default"
timeout -k 10 300 python bench.py --config C --steps 2 --warmup 1 --no-cpu > $OUT/bench_C.log 2>&1 || { tail -20 $OUT/bench_C.log; exit 1; }
for E in exp2 exp3; do
  echo "[$(date +%T)] C $E"
  GWAMD_DIAG=1 GWAMD_LIBRARY=claragenomicsanalysis_amd/lib/$E/libgwamd.so timeout -k 10 300 python bench.py --config C --steps 2 --warmup 1 --no-cpu > $OUT/bench_C_$E.log 2>&1
  rc=$?; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then tail -20 $OUT/bench_C_$E.log; exit 1; fi
done
echo "[$(date +%T)] done"
