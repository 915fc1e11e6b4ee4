#!/bin/bash
# round 5: anti-diagonal pass with the next step's LDS loads issued at the
# top of each step: banded parity, then C and B_banded
cd "$(dirname "$0")/../.." || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/r5i
mkdir -p $OUT
echo "[$(date +%T)] pytest banded"
timeout -k 10 900 python -u -m pytest tests/test_poa_gpu.py tests/test_poa_weights.py -k "band or anti or traceback_walk or persistent or config_c" -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_band.log 2>&1 || { tail -40 $OUT/pytest_band.log; exit 1; }
tail -2 $OUT/pytest_band.log
for C in C B_banded; do
  echo "[$(date +%T)] bench $C"
  timeout -k 10 300 python bench.py --config $C --steps 3 --warmup 1 --no-cpu > $OUT/bench_$C.log 2>&1 || { tail -20 $OUT/bench_$C.log; exit 1; }
done
echo "[$(date +%T)] done"
