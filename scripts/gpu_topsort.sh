#!/bin/bash
# Kahn sort with the single-successor run loop: POA parity tests, then
# config B and C bench lines (phase split shows the sort).
cd "$(dirname "$0")/.." || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/ts
mkdir -p $OUT
step() { echo "[$(date +%T)] $*"; }
step "pytest poa"
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "poa or band or cudapoa or spoa or msa or multibatch" > $OUT/pytest_poa.log 2>&1 || { tail -30 $OUT/pytest_poa.log; exit 1; }
tail -2 $OUT/pytest_poa.log
step "bench B"
timeout -k 10 300 python bench.py --config B --steps 10 --warmup 2 --no-cpu --no-secondary > $OUT/bench_B.log 2>&1 || { tail -20 $OUT/bench_B.log; exit 1; }
step "bench C"
timeout -k 10 300 python bench.py --config C --steps 5 --warmup 1 --no-cpu > $OUT/bench_C.log 2>&1 || { tail -20 $OUT/bench_C.log; exit 1; }
step done
