#!/bin/bash
# Round 3: forward-pass predecessor prefetch (LDS kernel) -- GPU tests, the
# default bench line, and config B with the prefetch off (A/B on one box).
cd "$(dirname "$0")/.." || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/r3v
mkdir -p $OUT
step() { echo "[$(date +%T)] $*"; }
step "pytest -m gpu"
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -3 $OUT/pytest_gpu.log
step "bench default"
timeout -k 10 400 python bench.py > $OUT/bench_default.log 2>&1 || { tail -20 $OUT/bench_default.log; exit 1; }
step "bench B, prefetch off"
GWAMD_FWD_PREFETCH=0 timeout -k 10 300 python bench.py --no-cpu --no-secondary > $OUT/bench_B_nopf.log 2>&1 || { tail -20 $OUT/bench_B_nopf.log; exit 1; }
step "bench B, prefetch on"
timeout -k 10 300 python bench.py --no-cpu --no-secondary > $OUT/bench_B_pf.log 2>&1 || { tail -20 $OUT/bench_B_pf.log; exit 1; }
step done
