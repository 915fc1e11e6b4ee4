#!/bin/bash
# round 5: the LDS kernel's 32-bit pass (parity at every shape, weights,
# persistent grid) and the F_int32_4k bench line
cd "$(dirname "$0")/../.." || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/r5c
mkdir -p $OUT
echo "[$(date +%T)] pytest int32"
timeout -k 10 900 python -u -m pytest tests/test_poa_gpu.py tests/test_poa_weights.py -k "int32 or weighted" -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_int32.log 2>&1 || { tail -40 $OUT/pytest_int32.log; exit 1; }
tail -2 $OUT/pytest_int32.log
echo "[$(date +%T)] bench F_int32_4k"
timeout -k 10 400 python bench.py --config F_int32_4k --steps 3 --warmup 1 > $OUT/bench_F.log 2>&1 || { tail -20 $OUT/bench_F.log; exit 1; }
tail -c 400 $OUT/bench_F.log
echo "[$(date +%T)] done"
