#!/bin/bash
# Round-2 final-tree check: GPU parity tests, smoke, default bench line and
# config C; stops at the first failing step.  Output under gpurun_out/r2d/.
cd "$(dirname "$0")/.." || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/r2d
mkdir -p $OUT
step() { echo "[$(date +%T)] $*"; }
step "pytest -m gpu"
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -3 $OUT/pytest_gpu.log
step "smoke"
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
step "bench default"
timeout -k 10 420 python bench.py > $OUT/bench_default.log 2>&1 || { tail -20 $OUT/bench_default.log; exit 1; }
step "bench C"
timeout -k 10 300 python bench.py --config C --steps 5 --warmup 1 > $OUT/bench_C.log 2>&1 || { tail -20 $OUT/bench_C.log; exit 1; }
step done
