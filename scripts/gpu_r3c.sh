#!/bin/bash
# Round 3, call c: GPU tests (tiled full-Myers backtrace), D_myers bench +
# kernel stats + HBM + SQ passes, full-Myers phase counters, banded 64k split
# (no-backtrace build), config B forward shapes and forward section timers.
cd "$(dirname "$0")/.." || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/r3c
mkdir -p $OUT
step() { echo "[$(date +%T)] $*"; }
step "pytest -m gpu"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
step "bench D_myers"
timeout -k 10 300 python bench.py --config D_myers --steps 3 --warmup 1 > $OUT/bench_D_myers.log 2>&1 || { tail -20 $OUT/bench_D_myers.log; exit 1; }
tail -c 400 $OUT/bench_D_myers.log
step "aln_prof myers"
timeout -k 10 300 python scripts/aln_prof.py 20000 myers > $OUT/alnprof_myers.log 2>&1 || { tail -5 $OUT/alnprof_myers.log; exit 1; }
cat $OUT/alnprof_myers.log
step "profile D_myers"
TAG=r3c_D_myers PROF_TIMEOUT=300 BENCH_ARGS="--config D_myers --steps 1 --warmup 1 --no-cpu" bash scripts/profile.sh > $OUT/prof_D_myers.log 2>&1 || { tail -20 $OUT/prof_D_myers.log; exit 1; }
step "sq D_myers"
TAG=r3c_D_myers PROF_TIMEOUT=300 BENCH_ARGS="--config D_myers --steps 1 --warmup 0 --no-cpu" bash scripts/pmc_sq.sh > $OUT/sq_D_myers.log 2>&1 || { tail -20 $OUT/sq_D_myers.log; exit 1; }
step "banded 64k without backtrace"
GWAMD_LIBRARY=$PWD/claragenomicsanalysis_amd/lib/exp/libgwamd.so timeout -k 10 300 python bench.py --config D_banded_64k --steps 1 --warmup 0 --no-cpu > $OUT/bench_D_banded_64k_nobt.log 2>&1
tail -c 300 $OUT/bench_D_banded_64k_nobt.log
for S in 8,2 4,4 8,4 16,4 8,3; do
  step "B shape $S"
  GWAMD_POA_LDS_SHAPE=$S timeout -k 10 200 python bench.py --config B --steps 5 --warmup 1 --no-cpu > $OUT/bench_B_$S.log 2>&1 || { tail -5 $OUT/bench_B_$S.log; exit 1; }
done
TAG=r3c bash scripts/gpu_fwdprof.sh > $OUT/fwdprof.log 2>&1 || { tail -5 $OUT/fwdprof.log; exit 1; }
cat $OUT/fwdprof.log
step done
