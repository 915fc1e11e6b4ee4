#!/bin/bash
# Round 3, final measurements (part 1): smoke, the default bench line, the
# other configs' lines, and rocprofv3 kernel stats + FETCH_SIZE / WRITE_SIZE
# passes for B, C, D, D_myers and E.
cd "$(dirname "$0")/.." || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/r3q
mkdir -p $OUT
step() { echo "[$(date +%T)] $*"; }
step "smoke"
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
step "bench default"
timeout -k 10 400 python bench.py > $OUT/bench_default.log 2>&1 || { tail -20 $OUT/bench_default.log; exit 1; }
for C in B_banded D_myers D_banded D_ukkonen; do
  step "bench $C"
  timeout -k 10 300 python bench.py --config $C --steps 3 --warmup 1 --no-secondary > $OUT/bench_$C.log 2>&1 || { tail -20 $OUT/bench_$C.log; exit 1; }
done
for C in D_100k D_myers_64k D_banded_64k B_banded_512 C_512; do
  step "bench $C"
  timeout -k 10 300 python bench.py --config $C --steps 1 --warmup 1 --no-cpu --no-secondary > $OUT/bench_$C.log 2>&1 || { tail -20 $OUT/bench_$C.log; exit 1; }
done
for C in B C D D_myers; do
  step "profile $C"
  TAG=r3q_$C PROF_TIMEOUT=300 BENCH_ARGS="--config $C --steps 2 --warmup 1 --no-cpu --no-secondary" bash scripts/profile.sh > $OUT/prof_$C.log 2>&1 || { tail -20 $OUT/prof_$C.log; exit 1; }
done
step "profile E"
TAG=r3q_E PROF_TIMEOUT=300 BENCH_ARGS="--config E --steps 2 --warmup 0 --no-cpu" bash scripts/profile.sh > $OUT/prof_E.log 2>&1 || { tail -20 $OUT/prof_E.log; exit 1; }
step done
