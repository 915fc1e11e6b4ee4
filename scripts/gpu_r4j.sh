#!/bin/bash
# Round 4: D_banded_64k sweep time alone (library built with
# -DGWAMD_ALN_NO_BACKTRACE into lib/nobt; parity is expected to fail there).
cd "$(dirname "$0")/.." || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/r4j
mkdir -p $OUT
step() { echo "[$(date +%T)] $*"; }
step "bench D_banded_64k no backtrace"
GWAMD_DIAG=1 GWAMD_LIBRARY=$PWD/claragenomicsanalysis_amd/lib/nobt/libgwamd.so timeout -k 10 300 python bench.py --config D_banded_64k --steps 3 --warmup 1 --no-cpu > $OUT/bench_nobt.log 2>&1; echo "rc $?"
step done
