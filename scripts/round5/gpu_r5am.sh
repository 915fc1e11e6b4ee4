#!/bin/bash
# round 5: D_ukkonen backtrace tile size sweep with the window walk
cd "$(dirname "$0")/../.." || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/${TAG:-r5am}
mkdir -p $OUT
for TB in ${TBS:-3072 4096 5120 6144 8192}; do
  echo "[$(date +%T)] D_ukkonen tile $TB"
  GWAMD_DIAG=1 GWAMD_UK_TILE_BYTES=$TB timeout -k 10 300 python bench.py --config D_ukkonen --steps 3 --warmup 1 --no-cpu > $OUT/bench_D_ukkonen_t$TB.log 2>&1 || { tail -20 $OUT/bench_D_ukkonen_t$TB.log; exit 1; }
done
echo "[$(date +%T)] done"
