#!/bin/bash
# Round 4: ukkonen_kernel backtrace tile size (LDS per workgroup -> resident
# pairs): parity with a 16 KiB tile, then D_ukkonen at 8 KiB (default), 12 KiB
# and 16 KiB tiles on one box (run 1: 8, 4, 2 KiB: 215.9k, 166.0k, 181.8k).
cd "$(dirname "$0")/.." || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/r4n
mkdir -p $OUT
step() { echo "[$(date +%T)] $*"; }
step "pytest ukkonen 16 KiB tile"
GWAMD_DIAG=1 GWAMD_UK_TILE_BYTES=16384 timeout -k 10 600 python -u -m pytest tests/test_aligner_gpu.py tests/test_aligner_long.py -m gpu -k "kkonen" -x -v --timeout 300 --timeout-method thread > $OUT/pytest_uk.log 2>&1 || { tail -30 $OUT/pytest_uk.log; exit 1; }
tail -2 $OUT/pytest_uk.log
for TB in 8192 12288 16384; do
step "bench D_ukkonen tile $TB"
GWAMD_DIAG=1 GWAMD_UK_TILE_BYTES=$TB timeout -k 10 300 python bench.py --config D_ukkonen --steps 5 --warmup 1 --no-cpu > $OUT/bench_uk_$TB.log 2>&1 || { tail -20 $OUT/bench_uk_$TB.log; exit 1; }
done
step done
