#!/bin/bash
# Round 3: strip-shaped traceback move windows (TbWin) -- GPU tests, then the
# default bench line with strips (default) and with 16 x 8 rectangles (A/B on
# one box).
cd "$(dirname "$0")/.." || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/${OUT_TAG:-r3t}
mkdir -p $OUT
step() { echo "[$(date +%T)] $*"; }
step "pytest -m gpu"
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -3 $OUT/pytest_gpu.log
step "bench default (strip windows)"
timeout -k 10 400 python bench.py > $OUT/bench_default.log 2>&1 || { tail -20 $OUT/bench_default.log; exit 1; }
step "bench default (rectangles)"
GWAMD_TB_WALK=rect timeout -k 10 400 python bench.py --no-cpu > $OUT/bench_rect.log 2>&1 || { tail -20 $OUT/bench_rect.log; exit 1; }
step done
