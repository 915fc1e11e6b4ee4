#!/bin/bash
# Round 3, call f: the original add restored (FIFO v2 kept), full Myers with
# patterns in HBM: GPU tests, B / C / D_myers lines, C sequential-add count.
cd "$(dirname "$0")/.." || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/r3f
mkdir -p $OUT
step() { echo "[$(date +%T)] $*"; }
step "pytest -m gpu"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
for C in B C D_myers; do
  step "bench $C"
  timeout -k 10 300 python bench.py --config $C --steps 5 --warmup 1 --no-cpu > $OUT/bench_$C.log 2>&1 || { tail -20 $OUT/bench_$C.log; exit 1; }
done
step "C band counters"
GWAMD_LIBRARY=$PWD/claragenomicsanalysis_amd/lib/bandprof/libgwamd.so timeout -k 10 300 python bench.py --config C --steps 1 --warmup 0 --no-cpu --no-secondary > $OUT/bench_C_bandprof.log 2>&1 || { tail -20 $OUT/bench_C_bandprof.log; exit 1; }
step done
