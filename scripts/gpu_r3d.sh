#!/bin/bash
# Round 3, call d: Kahn FIFO with the next pop's read issued alongside,
# line-aligned full-Myers rows: GPU tests, B / C / D_myers lines, D_myers HBM
# passes, topsort counters on C.
cd "$(dirname "$0")/.." || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/r3d
mkdir -p $OUT
step() { echo "[$(date +%T)] $*"; }
step "pytest -m gpu"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
for C in B C D_myers; do
  step "bench $C"
  timeout -k 10 300 python bench.py --config $C --steps 5 --warmup 1 --no-cpu > $OUT/bench_$C.log 2>&1 || { tail -20 $OUT/bench_$C.log; exit 1; }
  tail -c 250 $OUT/bench_$C.log; echo
done
step "aln_prof myers"
timeout -k 10 300 python scripts/aln_prof.py 20000 myers > $OUT/alnprof_myers.log 2>&1 || { tail -5 $OUT/alnprof_myers.log; exit 1; }
cat $OUT/alnprof_myers.log
step "profile D_myers"
TAG=r3d_D_myers PROF_TIMEOUT=300 BENCH_ARGS="--config D_myers --steps 1 --warmup 1 --no-cpu" bash scripts/profile.sh > $OUT/prof_D_myers.log 2>&1 || { tail -20 $OUT/prof_D_myers.log; exit 1; }
step "C topsort counters"
GWAMD_LIBRARY=$PWD/claragenomicsanalysis_amd/lib/tsprof/libgwamd.so timeout -k 10 300 python bench.py --config C --steps 1 --warmup 0 --no-cpu --no-secondary > $OUT/bench_C_tsprof.log 2>&1 || { tail -20 $OUT/bench_C_tsprof.log; exit 1; }
step done
