#!/bin/bash
# Round 3: forward-pass section timers of config B (diagnostic builds
# lib/prof = wave 0, lib/prof1 = wave 1; phase slots hold cycles / 1e5).
cd "$(dirname "$0")/.." || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/r3u
mkdir -p $OUT
step() { echo "[$(date +%T)] $*"; }
for W in prof prof1; do
  step "bench B with lib/$W"
  GWAMD_LIBRARY=claragenomicsanalysis_amd/lib/$W/libgwamd.so timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu --no-secondary > $OUT/bench_$W.log 2>&1 || { tail -20 $OUT/bench_$W.log; exit 1; }
done
step done
