#!/bin/bash
# Round 4, first check of the tree: GPU tests (ring-mode Kahn sort, banded-
# Myers HBM-state counter, wide Ukkonen), the default bench line and the
# Ukkonen lines.
cd "$(dirname "$0")/.." || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/r4a
mkdir -p $OUT
step() { echo "[$(date +%T)] $*"; }
step "pytest gpu"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -3 $OUT/pytest_gpu.log
for C in D_ukkonen_wide_16k D_ukkonen_64k D_ukkonen; do
  step "bench $C"
  timeout -k 10 300 python bench.py --config $C --steps 3 --warmup 1 > $OUT/bench_$C.log 2>&1 || { tail -20 $OUT/bench_$C.log; exit 1; }
done
step "bench default"
timeout -k 10 400 python bench.py > $OUT/bench_default.log 2>&1 || { tail -20 $OUT/bench_default.log; exit 1; }
step done
