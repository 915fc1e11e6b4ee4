#!/bin/bash
# Round 3, call b: GPU tests (multibatch skip/timing, banded_ad persistent grid),
# smoke, the new default bench line (B + D, C, E), full-Myers phase counters,
# kernel stats + HBM passes for D_myers, SQ passes for D (hm_kernel) and D_myers.
cd "$(dirname "$0")/.." || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/r3b
mkdir -p $OUT
step() { echo "[$(date +%T)] $*"; }
step "pytest -m gpu"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
step "smoke"
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
step "bench default"
timeout -k 10 600 python bench.py > $OUT/bench_default.log 2>&1 || { tail -20 $OUT/bench_default.log; exit 1; }
tail -c 600 $OUT/bench_default.log
for C in D_100k D_myers_64k D_banded_64k; do
  step "bench $C"
  timeout -k 10 300 python bench.py --config $C --steps 1 --warmup 1 --no-cpu > $OUT/bench_$C.log 2>&1 || { tail -20 $OUT/bench_$C.log; exit 1; }
  tail -c 300 $OUT/bench_$C.log
done
step "aln_prof myers"
timeout -k 10 300 python scripts/aln_prof.py 20000 myers > $OUT/alnprof_myers.log 2>&1 || { tail -5 $OUT/alnprof_myers.log; exit 1; }
cat $OUT/alnprof_myers.log
step "profile D_myers"
TAG=r3_D_myers PROF_TIMEOUT=300 BENCH_ARGS="--config D_myers --steps 1 --warmup 1 --no-cpu" bash scripts/profile.sh > $OUT/prof_D_myers.log 2>&1 || { tail -20 $OUT/prof_D_myers.log; exit 1; }
step "sq D"
TAG=r3_D PROF_TIMEOUT=300 BENCH_ARGS="--config D --steps 1 --warmup 0 --no-cpu" bash scripts/pmc_sq.sh > $OUT/sq_D.log 2>&1 || { tail -20 $OUT/sq_D.log; exit 1; }
step "sq D_myers"
TAG=r3_D_myers PROF_TIMEOUT=300 BENCH_ARGS="--config D_myers --steps 1 --warmup 0 --no-cpu" bash scripts/pmc_sq.sh > $OUT/sq_D_myers.log 2>&1 || { tail -20 $OUT/sq_D_myers.log; exit 1; }
step done1
for P in tsprof bandprof; do
  step "C counters $P"
  GWAMD_LIBRARY=$PWD/claragenomicsanalysis_amd/lib/$P/libgwamd.so timeout -k 10 300 python bench.py --config C --steps 1 --warmup 0 --no-cpu --no-secondary > $OUT/bench_C_$P.log 2>&1 || { tail -20 $OUT/bench_C_$P.log; exit 1; }
done
step done2
