#!/bin/bash
# Round 4: typed pointers in the out-of-line traceback and split sweeps.  All
# GPU tests, then B, C and D lines.
cd "$(dirname "$0")/.." || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/r4c
mkdir -p $OUT
step() { echo "[$(date +%T)] $*"; }
step "pytest gpu"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
for C in B C D; do
  step "bench $C"
  timeout -k 10 400 python bench.py --config $C --steps 5 --warmup 1 --no-cpu > $OUT/bench_$C.log 2>&1 || { tail -20 $OUT/bench_$C.log; exit 1; }
done
step done
