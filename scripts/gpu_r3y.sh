#!/bin/bash
# Round 3 (re-entry), final measurements part 2: SQ counter passes for B, C
# and E of this tree.
cd "$(dirname "$0")/.." || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/r3y
mkdir -p $OUT
step() { echo "[$(date +%T)] $*"; }
for C in B C; do
  step "sq $C"
  TAG=r3y_$C PROF_TIMEOUT=300 BENCH_ARGS="--config $C --steps 1 --warmup 0 --no-cpu --no-secondary" bash scripts/pmc_sq.sh > $OUT/sq_$C.log 2>&1 || { tail -20 $OUT/sq_$C.log; exit 1; }
done
step "sq E"
TAG=r3y_E PROF_TIMEOUT=300 BENCH_ARGS="--config E --steps 2 --warmup 0 --no-cpu" bash scripts/pmc_sq.sh > $OUT/sq_E.log 2>&1 || { tail -20 $OUT/sq_E.log; exit 1; }
step done
