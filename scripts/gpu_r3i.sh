#!/bin/bash
# Round 3, call i: LDS band kernel at band width 512 (8 cells per lane): its
# parity tests first, then the whole GPU suite, the bw 512 lines, and the SQ
# counter passes of B, C, E, D_myers for the final profiles.
cd "$(dirname "$0")/.." || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/r3i
mkdir -p $OUT
step() { echo "[$(date +%T)] $*"; }
step "pytest bw 512"
timeout -k 10 300 python -u -m pytest tests/test_poa_gpu.py -m gpu -x -v -k "512" --timeout 150 --timeout-method thread > $OUT/pytest_512.log 2>&1 || { tail -30 $OUT/pytest_512.log; exit 1; }
tail -2 $OUT/pytest_512.log
step "pytest -m gpu"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
for C in B_banded_512 C_512 B_banded C; do
  step "bench $C"
  timeout -k 10 300 python bench.py --config $C --steps 3 --warmup 1 --no-cpu > $OUT/bench_$C.log 2>&1 || { tail -20 $OUT/bench_$C.log; exit 1; }
done
for C in B C D_myers; do
  step "sq $C"
  TAG=r3i_$C PROF_TIMEOUT=300 BENCH_ARGS="--config $C --steps 1 --warmup 0 --no-cpu --no-secondary" bash scripts/pmc_sq.sh > $OUT/sq_$C.log 2>&1 || { tail -20 $OUT/sq_$C.log; exit 1; }
done
step "sq E"
TAG=r3i_E PROF_TIMEOUT=300 BENCH_ARGS="--config E --steps 2 --warmup 0 --no-cpu" bash scripts/pmc_sq.sh > $OUT/sq_E.log 2>&1 || { tail -20 $OUT/sq_E.log; exit 1; }
step done
