#!/bin/bash
# Round-end measurement on one GPU: parity tests, bench lines for every
# config, rocprofv3 kernel stats + HBM counters for configs B and D.
# Output under gpurun_out/measure_<TAG>/.  Stops at the first failing step.
cd "$(dirname "$0")/.." || exit 1
TAG=${TAG:-r1}
OUT=gpurun_out/measure_$TAG
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
step() { echo "[$(date +%T)] $*"; }
step "pytest -m gpu"
timeout -k 10 600 python -m pytest tests -m gpu -q > $OUT/pytest_gpu.log 2>&1; rc=$?
tail -3 $OUT/pytest_gpu.log
if [ $rc -ne 0 ]; then echo "pytest rc=$rc"; exit $rc; fi
for C in B B_banded C D D_myers D_banded D_ukkonen; do
  step "bench $C"
  timeout -k 10 400 python bench.py --config $C --steps ${STEPS:-5} --warmup 1 > $OUT/bench_$C.log 2>&1 || { echo "bench $C failed"; tail -20 $OUT/bench_$C.log; exit 1; }
  tail -1 $OUT/bench_$C.log | cut -c1-160
done
if [ -z "$SKIP_PROF" ]; then
  step "profile B"
  TAG=${TAG}_B BENCH_ARGS="--config B --steps 2 --warmup 1 --no-cpu" bash scripts/profile.sh > $OUT/prof_B.log 2>&1 || { tail -20 $OUT/prof_B.log; exit 1; }
  step "profile B_banded"
  TAG=${TAG}_B_banded BENCH_ARGS="--config B_banded --steps 2 --warmup 1 --no-cpu" bash scripts/profile.sh > $OUT/prof_B_banded.log 2>&1 || { tail -20 $OUT/prof_B_banded.log; exit 1; }
  step "profile C"
  TAG=${TAG}_C BENCH_ARGS="--config C --steps 2 --warmup 1 --no-cpu" bash scripts/profile.sh > $OUT/prof_C.log 2>&1 || { tail -20 $OUT/prof_C.log; exit 1; }
  step "profile D"
  TAG=${TAG}_D BENCH_ARGS="--config D --steps 2 --warmup 1 --no-cpu" bash scripts/profile.sh > $OUT/prof_D.log 2>&1 || { tail -20 $OUT/prof_D.log; exit 1; }
fi
step done
