#!/bin/bash
# round 5: config B with 3 and 4 waves per window (LDS kernel shapes)
cd "$(dirname "$0")/../.." || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/r5u
mkdir -p $OUT
for SH in 8,2 8,3 8,4 4,4; do
  echo "[$(date +%T)] bench B shape $SH"
  GWAMD_DIAG=1 GWAMD_POA_LDS_SHAPE=$SH timeout -k 10 300 python bench.py --config B --steps 3 --warmup 1 --no-cpu > $OUT/bench_B_$SH.log 2>&1 || { tail -20 $OUT/bench_B_$SH.log; exit 1; }
done
echo "[$(date +%T)] done"
