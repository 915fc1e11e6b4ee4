#!/bin/bash
# Round 3: 32 x 4 traceback strips -- walk-mode parity tests, then B and C
# with 16 x 8 strips (default) and 32 x 4 strips (A/B on one box).
cd "$(dirname "$0")/.." || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/r3w
mkdir -p $OUT
step() { echo "[$(date +%T)] $*"; }
step "pytest -m gpu"
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -3 $OUT/pytest_gpu.log
for W in default strip32; do
  for C in B C; do
    step "bench $C, walk $W"
    GWAMD_TB_WALK=$W timeout -k 10 300 python bench.py --config $C --steps 5 --warmup 1 --no-cpu --no-secondary > $OUT/bench_${C}_$W.log 2>&1 || { tail -20 $OUT/bench_${C}_$W.log; exit 1; }
  done
done
step done
