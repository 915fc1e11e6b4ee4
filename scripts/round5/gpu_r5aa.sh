#!/bin/bash
# round 5: SQ counters of ukkonen_kernel on D_ukkonen_64k, whole kernel and
# forward sweep alone (no-backtrace build), to split instructions and cycles
cd "$(dirname "$0")/../.." || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/r5aa
mkdir -p $OUT
echo "[$(date +%T)] sq whole"
TAG=r5aa_Duk64 PROF_TIMEOUT=200 BENCH_ARGS="--config D_ukkonen_64k --steps 1 --warmup 0 --no-cpu" bash scripts/pmc_sq.sh > $OUT/sq.log 2>&1 || { tail -20 $OUT/sq.log; exit 1; }
echo "[$(date +%T)] sq forward only"
ALLOW_FAIL=1 GWAMD_DIAG=1 GWAMD_LIBRARY=$PWD/claragenomicsanalysis_amd/lib/exp5/libgwamd.so TAG=r5aa_Duk64_fwd PROF_TIMEOUT=200 BENCH_ARGS="--config D_ukkonen_64k --steps 1 --warmup 0 --no-cpu" bash scripts/pmc_sq.sh > $OUT/sq_fwd.log 2>&1
echo "[$(date +%T)] done"
