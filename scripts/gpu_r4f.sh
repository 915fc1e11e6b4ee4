#!/bin/bash
# Round 4: anti-diagonal band pass out of line with global-typed pointers, paired Kahn pops:
# banded parity tests, then C and B_banded lines.
cd "$(dirname "$0")/.." || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/r4f
mkdir -p $OUT
step() { echo "[$(date +%T)] $*"; }
step "pytest poa gpu"
timeout -k 10 600 python -u -m pytest tests/test_poa_gpu.py tests/test_poa_multibatch.py -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/pytest_poa.log 2>&1 || { tail -30 $OUT/pytest_poa.log; exit 1; }
tail -2 $OUT/pytest_poa.log
for C in C B_banded B; do
  step "bench $C"
  timeout -k 10 300 python bench.py --config $C --steps 5 --warmup 1 --no-cpu > $OUT/bench_$C.log 2>&1 || { tail -20 $OUT/bench_$C.log; exit 1; }
done
step done
