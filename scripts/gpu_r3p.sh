#!/bin/bash
# Round 3, call p: SQ counters of the banded Myers kernel at 65,536 bp.
cd "$(dirname "$0")/.." || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/r3p
mkdir -p $OUT
step() { echo "[$(date +%T)] $*"; }
step "sq D_banded_64k"
TAG=r3p_D_banded_64k PROF_TIMEOUT=200 BENCH_ARGS="--config D_banded_64k --steps 1 --warmup 0 --no-cpu --no-secondary" bash scripts/pmc_sq.sh > $OUT/sq.log 2>&1 || { tail -20 $OUT/sq.log; exit 1; }
step done
