#!/bin/bash
# Round 4: Kahn chain runs A/B (lib/var_nochain built with -DGWAMD_NO_TOPSORT_CHAINS)
# on configs B and C, same box.
cd "$(dirname "$0")/.." || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/r4d
mkdir -p $OUT
step() { echo "[$(date +%T)] $*"; }
for C in B C; do
  step "bench $C chains"
  timeout -k 10 300 python bench.py --config $C --steps 5 --warmup 1 --no-cpu > $OUT/bench_${C}_chain.log 2>&1 || { tail -20 $OUT/bench_${C}_chain.log; exit 1; }
  step "bench $C nochain"
  GWAMD_DIAG=1 GWAMD_LIBRARY=claragenomicsanalysis_amd/lib/var_nochain/libgwamd.so timeout -k 10 300 python bench.py --config $C --steps 5 --warmup 1 --no-cpu > $OUT/bench_${C}_nochain.log 2>&1 || { tail -20 $OUT/bench_${C}_nochain.log; exit 1; }
done
step done
