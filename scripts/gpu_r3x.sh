#!/bin/bash
# Round 3 (re-entry), final measurements part 1 for this tree: smoke, the
# default bench line, the other configs' lines, and rocprofv3 kernel stats +
# FETCH_SIZE / WRITE_SIZE passes for B, C and E (the aligner kernels did not
# change since profiles/r3q_D*).
cd "$(dirname "$0")/.." || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/r3x
mkdir -p $OUT
step() { echo "[$(date +%T)] $*"; }
step "smoke"
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
step "bench default"
timeout -k 10 400 python bench.py > $OUT/bench_default.log 2>&1 || { tail -20 $OUT/bench_default.log; exit 1; }
for C in B_banded; do
  step "bench $C"
  timeout -k 10 300 python bench.py --config $C --steps 3 --warmup 1 --no-secondary > $OUT/bench_$C.log 2>&1 || { tail -20 $OUT/bench_$C.log; exit 1; }
done
for C in B_banded_512 C_512; do
  step "bench $C"
  timeout -k 10 300 python bench.py --config $C --steps 1 --warmup 1 --no-cpu --no-secondary > $OUT/bench_$C.log 2>&1 || { tail -20 $OUT/bench_$C.log; exit 1; }
done
for C in B C; do
  step "profile $C"
  TAG=r3x_$C PROF_TIMEOUT=300 BENCH_ARGS="--config $C --steps 2 --warmup 1 --no-cpu --no-secondary" bash scripts/profile.sh > $OUT/prof_$C.log 2>&1 || { tail -20 $OUT/prof_$C.log; exit 1; }
done
step "profile E"
TAG=r3x_E PROF_TIMEOUT=300 BENCH_ARGS="--config E --steps 2 --warmup 0 --no-cpu" bash scripts/profile.sh > $OUT/prof_E.log 2>&1 || { tail -20 $OUT/prof_E.log; exit 1; }
step done
