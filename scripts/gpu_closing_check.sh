#!/bin/bash
# Closing check of the tree on one GPU box: all GPU tests, smoke, the default
# bench line, kernel stats + HBM passes and SQ counters for the configs in
# PROFILE (default "B C D"), and the bench lines of EXTRA configs.
#   TAG=r5a bash scripts/gpu_closing_check.sh
# Every GPU step runs under its own time limit; the first failure ends the run.
cd "$(dirname "$0")/.." || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0
TAG=${TAG:-check}
OUT=gpurun_out/$TAG
mkdir -p $OUT
step() { echo "[$(date +%T)] $*"; }
if [ -z "$SKIP_TESTS" ]; then
  step "pytest -m gpu"
  timeout -k 10 ${TEST_TIMEOUT:-900} python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread ${PYTEST_ARGS} > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
  tail -2 $OUT/pytest_gpu.log
  step "smoke"
  timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
fi
if [ -z "$SKIP_BENCH" ]; then
  step "bench default"
  timeout -k 10 500 python bench.py > $OUT/bench_default.log 2>&1 || { tail -20 $OUT/bench_default.log; exit 1; }
  tail -c 600 $OUT/bench_default.log
fi
for C in $EXTRA; do
  step "bench $C"
  timeout -k 10 400 python bench.py --config $C --steps 3 --warmup 1 > $OUT/bench_$C.log 2>&1 || { tail -20 $OUT/bench_$C.log; exit 1; }
done
for C in ${PROFILE-B C D}; do
  step "profile $C"
  TAG=${TAG}_$C PROF_TIMEOUT=300 BENCH_ARGS="--config $C --steps 2 --warmup 1 --no-cpu --no-secondary" bash scripts/profile.sh > $OUT/prof_$C.log 2>&1 || { tail -20 $OUT/prof_$C.log; exit 1; }
  step "sq $C"
  TAG=${TAG}_$C PROF_TIMEOUT=300 BENCH_ARGS="--config $C --steps 1 --warmup 0 --no-cpu --no-secondary" bash scripts/pmc_sq.sh > $OUT/sq_$C.log 2>&1 || { tail -20 $OUT/sq_$C.log; exit 1; }
done
step done
