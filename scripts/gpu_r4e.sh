#!/bin/bash
# Round 4 closing check of the tree: all GPU tests, smoke, the default bench
# line, kernel stats + HBM passes for B and C, SQ counters for B, and the
# lines of the global-memory kernel's shapes and the wide Ukkonen.
cd "$(dirname "$0")/.." || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/r4e
mkdir -p $OUT
step() { echo "[$(date +%T)] $*"; }
step "pytest -m gpu"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
step "smoke"
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
step "bench default"
timeout -k 10 500 python bench.py > $OUT/bench_default.log 2>&1 || { tail -20 $OUT/bench_default.log; exit 1; }
for C in B_banded_384 B_banded_1024 F_int32_4k; do
  step "bench $C"
  timeout -k 10 400 python bench.py --config $C --steps 3 --warmup 1 > $OUT/bench_$C.log 2>&1 || { tail -20 $OUT/bench_$C.log; exit 1; }
done
for C in B C; do
  step "profile $C"
  TAG=r4e_$C PROF_TIMEOUT=300 BENCH_ARGS="--config $C --steps 2 --warmup 1 --no-cpu --no-secondary" bash scripts/profile.sh > $OUT/prof_$C.log 2>&1 || { tail -20 $OUT/prof_$C.log; exit 1; }
done
step "sq B"
TAG=r4e_B PROF_TIMEOUT=300 BENCH_ARGS="--config B --steps 1 --warmup 0 --no-cpu --no-secondary" bash scripts/pmc_sq.sh > $OUT/sq_B.log 2>&1 || { tail -20 $OUT/sq_B.log; exit 1; }
step done
