#!/bin/bash
# Round 4 final closing check: all GPU tests, smoke, the default bench line
# (B + secondary D, C, E), D_banded_64k, kernel stats + HBM passes of D.
cd "$(dirname "$0")/.." || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/r4m
mkdir -p $OUT
step() { echo "[$(date +%T)] $*"; }
step "pytest -m gpu"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
step "smoke"
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
step "bench default"
timeout -k 10 500 python bench.py > $OUT/bench_default.log 2>&1 || { tail -20 $OUT/bench_default.log; exit 1; }
step "bench D_banded_64k"
timeout -k 10 300 python bench.py --config D_banded_64k --steps 3 --warmup 1 > $OUT/bench_D_banded_64k.log 2>&1 || { tail -20 $OUT/bench_D_banded_64k.log; exit 1; }
step "profile D"
TAG=r4m_D PROF_TIMEOUT=300 BENCH_ARGS="--config D --steps 2 --warmup 1 --no-cpu --no-secondary" bash scripts/profile.sh > $OUT/prof_D.log 2>&1 || { tail -20 $OUT/prof_D.log; exit 1; }
step done
