#!/bin/bash
# Round-2 final measurement: GPU parity tests, smoke, the default bench line
# (B + secondary D, E), config C, rocprofv3 kernel stats + HBM counter passes
# for B and C, SQ counter passes for B and C.  Output under gpurun_out/r2f/
# and gpurun_out/prof_r2f_*; stops at the first failing step.
cd "$(dirname "$0")/.." || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/r2f
mkdir -p $OUT
step() { echo "[$(date +%T)] $*"; }
step "pytest -m gpu"
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
step "smoke"
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
step "bench default"
timeout -k 10 420 python bench.py > $OUT/bench_default.log 2>&1 || { tail -20 $OUT/bench_default.log; exit 1; }
for C in C B_banded; do
  step "bench $C"
  timeout -k 10 300 python bench.py --config $C --steps 5 --warmup 1 > $OUT/bench_$C.log 2>&1 || { tail -20 $OUT/bench_$C.log; exit 1; }
done
for C in B C; do
  step "profile $C"
  TAG=r2f_$C BENCH_ARGS="--config $C --steps 2 --warmup 1 --no-cpu --no-secondary" bash scripts/profile.sh > $OUT/prof_$C.log 2>&1 || { tail -20 $OUT/prof_$C.log; exit 1; }
done
for C in B C; do
  step "sq $C"
  TAG=r2f_$C BENCH_ARGS="--config $C --steps 1 --warmup 0 --no-cpu --no-secondary" bash scripts/pmc_sq.sh > $OUT/sq_$C.log 2>&1 || { tail -20 $OUT/sq_$C.log; exit 1; }
done
step done
