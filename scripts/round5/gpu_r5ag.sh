#!/bin/bash
# round 5: D_banded backtrace tile size (LDS bytes) sweep
cd "$(dirname "$0")/../.." || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/r5ag
mkdir -p $OUT
for TB in 3072 3584 4096 6144; do
  echo "[$(date +%T)] D_banded tile $TB"
  GWAMD_DIAG=1 GWAMD_BAND_TILE_BYTES=$TB timeout -k 10 300 python bench.py --config D_banded --steps 3 --warmup 1 --no-cpu > $OUT/bench_D_banded_t$TB.log 2>&1 || { tail -20 $OUT/bench_D_banded_t$TB.log; exit 1; }
done
echo "[$(date +%T)] done"
