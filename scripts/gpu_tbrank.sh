#!/bin/bash
# Pointer-doubling traceback walk: POA parity tests with it (default), then
# config B and C bench lines with it and with the scalar walk, same box.
cd "$(dirname "$0")/.." || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/tbr
mkdir -p $OUT
step() { echo "[$(date +%T)] $*"; }
step "pytest poa"
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "poa or band or cudapoa or spoa or msa" > $OUT/pytest_poa.log 2>&1 || { tail -30 $OUT/pytest_poa.log; exit 1; }
tail -2 $OUT/pytest_poa.log
for W in rank scalar; do
  step "bench B $W"
  GWAMD_TB_WALK=$W timeout -k 10 300 python bench.py --config B --steps 10 --warmup 2 --no-cpu --no-secondary > $OUT/bench_B_$W.log 2>&1 || { tail -20 $OUT/bench_B_$W.log; exit 1; }
  step "bench C $W"
  GWAMD_TB_WALK=$W timeout -k 10 300 python bench.py --config C --steps 5 --warmup 1 --no-cpu > $OUT/bench_C_$W.log 2>&1 || { tail -20 $OUT/bench_C_$W.log; exit 1; }
done
step done
