#!/bin/bash
# Kahn sort with the queued-word ring for large graphs: POA parity tests,
# config C and B bench lines, then config C kernel stats + HBM passes.
cd "$(dirname "$0")/.." || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/ts2
mkdir -p $OUT
step() { echo "[$(date +%T)] $*"; }
step "pytest poa"
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "poa or band or cudapoa or spoa or msa or multibatch" > $OUT/pytest_poa.log 2>&1 || { tail -30 $OUT/pytest_poa.log; exit 1; }
tail -2 $OUT/pytest_poa.log
step "bench C"
timeout -k 10 300 python bench.py --config C --steps 5 --warmup 1 > $OUT/bench_C.log 2>&1 || { tail -20 $OUT/bench_C.log; exit 1; }
step "bench default"
timeout -k 10 420 python bench.py > $OUT/bench_default.log 2>&1 || { tail -20 $OUT/bench_default.log; exit 1; }
step "profile C"
TAG=r2g_C BENCH_ARGS="--config C --steps 2 --warmup 1 --no-cpu --no-secondary" bash scripts/profile.sh > $OUT/prof_C.log 2>&1 || { tail -20 $OUT/prof_C.log; exit 1; }
step done
