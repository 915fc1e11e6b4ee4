#!/bin/bash
# Round-2 measurement on one GPU: the default bench line (B + secondary D, E),
# every other config, rocprofv3 kernel stats + HBM counter passes for B, C, D,
# the kernel trace of E, SQ counter passes for B and C.  Output under
# gpurun_out/r2m/ (summarised into profiles/ by scripts/summarize_profile.py
# and scripts/sq_summary.py afterwards).  Stops at the first failing step.
cd "$(dirname "$0")/.." || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/r2m
mkdir -p $OUT
step() { echo "[$(date +%T)] $*"; }
step "bench default"
timeout -k 10 420 python bench.py > $OUT/bench_default.log 2>&1 || { tail -20 $OUT/bench_default.log; exit 1; }
for C in C B_banded D_myers D_banded D_ukkonen; do
  step "bench $C"
  timeout -k 10 400 python bench.py --config $C --steps ${STEPS:-5} --warmup 1 > $OUT/bench_$C.log 2>&1 || { echo "bench $C failed"; tail -20 $OUT/bench_$C.log; exit 1; }
done
for C in B C D; do
  step "profile $C"
  TAG=r2_$C BENCH_ARGS="--config $C --steps 2 --warmup 1 --no-cpu --no-secondary" bash scripts/profile.sh > $OUT/prof_$C.log 2>&1 || { tail -20 $OUT/prof_$C.log; exit 1; }
done
step "trace E"
TAG=r2_E COUNTERS=" " BENCH_ARGS="--config E --steps 4 --warmup 0 --no-cpu" bash scripts/profile.sh > $OUT/prof_E.log 2>&1 || { tail -20 $OUT/prof_E.log; exit 1; }
for C in B C; do
  step "sq $C"
  TAG=r2_$C BENCH_ARGS="--config $C --steps 1 --warmup 0 --no-cpu --no-secondary" bash scripts/pmc_sq.sh > $OUT/sq_$C.log 2>&1 || { tail -20 $OUT/sq_$C.log; exit 1; }
done
step done
