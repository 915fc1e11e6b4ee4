#!/bin/bash
# round 5: band kernel at every band width up to 1,024 (parity + bench lines),
# then refresh the C / D / E evidence the bench lines cite (kernel stats, HBM
# passes and SQ counters of the current kernels)
cd "$(dirname "$0")/../.." || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/r5b
mkdir -p $OUT
echo "[$(date +%T)] pytest banded"
timeout -k 10 900 python -u -m pytest tests/test_poa_gpu.py -k "banded or band_anti or traceback_walk or persistent" -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_band.log 2>&1 || { tail -30 $OUT/pytest_band.log; exit 1; }
tail -2 $OUT/pytest_band.log
for C in B_banded_384 B_banded_1024 B_banded B_banded_512; do
  echo "[$(date +%T)] bench $C"
  timeout -k 10 400 python bench.py --config $C --steps 3 --warmup 1 > $OUT/bench_$C.log 2>&1 || { tail -20 $OUT/bench_$C.log; exit 1; }
done
SKIP_TESTS=1 SKIP_BENCH=1 PROFILE="C D" TAG=r5b bash scripts/gpu_closing_check.sh || exit 1
echo "[$(date +%T)] profile E"
TAG=r5b_E PROF_TIMEOUT=300 BENCH_ARGS="--config E --steps 2 --warmup 0 --no-cpu" bash scripts/profile.sh > $OUT/prof_E.log 2>&1 || { tail -20 $OUT/prof_E.log; exit 1; }
echo "[$(date +%T)] done"
