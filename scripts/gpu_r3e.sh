#!/bin/bash
# Round 3, call e: branch-free single-successor Kahn pops, full-Myers tile 4x64
# and 64 GiB workspace (+ patterns-in-HBM experiment): GPU tests, B / C /
# D_myers lines, topsort counters on C and B, bw=512 lines.
cd "$(dirname "$0")/.." || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/r3e
mkdir -p $OUT
step() { echo "[$(date +%T)] $*"; }
step "pytest -m gpu"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
for C in B C D_myers; do
  step "bench $C"
  timeout -k 10 300 python bench.py --config $C --steps 5 --warmup 1 --no-cpu > $OUT/bench_$C.log 2>&1 || { tail -20 $OUT/bench_$C.log; exit 1; }
done
step "bench D_myers (patterns in HBM)"
GWAMD_MYERS_LONG=1 timeout -k 10 300 python bench.py --config D_myers --steps 5 --warmup 1 --no-cpu > $OUT/bench_D_myers_long.log 2>&1 || { tail -20 $OUT/bench_D_myers_long.log; exit 1; }
for C in C B; do
  step "topsort counters $C"
  GWAMD_LIBRARY=$PWD/claragenomicsanalysis_amd/lib/tsprof/libgwamd.so timeout -k 10 300 python bench.py --config $C --steps 1 --warmup 0 --no-cpu --no-secondary > $OUT/bench_${C}_tsprof.log 2>&1 || { tail -20 $OUT/bench_${C}_tsprof.log; exit 1; }
done
for C in B_banded_512 C_512; do
  step "bench $C"
  timeout -k 10 400 python bench.py --config $C --steps 2 --warmup 1 --no-cpu > $OUT/bench_$C.log 2>&1 || { tail -20 $OUT/bench_$C.log; exit 1; }
done
step done
