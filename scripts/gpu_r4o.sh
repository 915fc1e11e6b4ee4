#!/bin/bash
# Round 4: banded Myers tile / chunk-state LDS for short pairs (D_banded):
# 4 KiB (default) against 2 KiB (more resident pairs per CU), parity at 2 KiB.
cd "$(dirname "$0")/.." || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/r4o
mkdir -p $OUT
step() { echo "[$(date +%T)] $*"; }
step "pytest banded 2 KiB"
GWAMD_DIAG=1 GWAMD_BAND_TILE_BYTES=2048 timeout -k 10 600 python -u -m pytest tests/test_aligner_gpu.py -m gpu -k "banded" -x -v --timeout 300 --timeout-method thread > $OUT/pytest_b.log 2>&1 || { tail -30 $OUT/pytest_b.log; exit 1; }
tail -2 $OUT/pytest_b.log
for TB in 4096 2048 4096; do
step "bench D_banded tile $TB"
GWAMD_DIAG=1 GWAMD_BAND_TILE_BYTES=$TB timeout -k 10 300 python bench.py --config D_banded --steps 5 --warmup 1 --no-cpu > $OUT/bench_b_$TB.log 2>&1 || { tail -20 $OUT/bench_b_$TB.log; exit 1; }
done
step done
