#!/bin/bash
# Round 4: configs B and C after removing the Kahn chain runs (they skipped
# almost nothing on mature graphs: 5 of 2,034 nodes at B, 57 of 42,099 at C).
cd "$(dirname "$0")/.." || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/r4d
mkdir -p $OUT
step() { echo "[$(date +%T)] $*"; }
for C in B C; do
  step "bench $C"
  timeout -k 10 300 python bench.py --config $C --steps 5 --warmup 1 --no-cpu > $OUT/bench_${C}.log 2>&1 || { tail -20 $OUT/bench_${C}.log; exit 1; }
done
step done
