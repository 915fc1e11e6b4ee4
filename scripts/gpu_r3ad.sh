#!/bin/bash
# Round 3: strip rows above the slope line (GWAMD_TB_ABOVE) -- walk-mode parity
# with a non-default offset, then B and C per offset (A/B on one box).
cd "$(dirname "$0")/.." || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/r3ad
mkdir -p $OUT
step() { echo "[$(date +%T)] $*"; }
step "pytest -m gpu (default offset)"
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
step "walk-mode parity, 4 rows above"
GWAMD_TB_ABOVE=4 timeout -k 10 600 python -u -m pytest tests/test_poa_gpu.py -m gpu -x -q -k "walk_modes" --timeout 120 --timeout-method thread > $OUT/pytest_ab4.log 2>&1 || { tail -30 $OUT/pytest_ab4.log; exit 1; }
tail -2 $OUT/pytest_ab4.log
for A in 2 1 3 4; do
  for C in B C; do
    step "bench $C above $A"
    GWAMD_TB_ABOVE=$A timeout -k 10 300 python bench.py --config $C --steps 5 --warmup 1 --no-cpu --no-secondary > $OUT/bench_${C}_ab$A.log 2>&1 || { tail -20 $OUT/bench_${C}_ab$A.log; exit 1; }
  done
done
step done
