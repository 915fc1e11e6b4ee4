#!/bin/bash
# Round 4: Hirschberg-Myers split scores in LDS up to 2,048 columns (variant
# library lib/s2048) against the default 512: HM parity on the variant, then
# the D line with each library on the same box.
cd "$(dirname "$0")/.." || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/r4k
mkdir -p $OUT
V=$PWD/claragenomicsanalysis_amd/lib/s2048/libgwamd.so
step() { echo "[$(date +%T)] $*"; }
step "pytest aligner (s2048)"
GWAMD_DIAG=1 GWAMD_LIBRARY=$V timeout -k 10 600 python -u -m pytest tests/test_aligner_gpu.py tests/test_aligner_long.py -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_aln.log 2>&1 || { tail -30 $OUT/pytest_aln.log; exit 1; }
tail -2 $OUT/pytest_aln.log
step "bench D default"
timeout -k 10 300 python bench.py --config D --steps 5 --warmup 1 --no-cpu > $OUT/bench_D.log 2>&1 || { tail -20 $OUT/bench_D.log; exit 1; }
step "bench D s2048"
GWAMD_DIAG=1 GWAMD_LIBRARY=$V timeout -k 10 300 python bench.py --config D --steps 5 --warmup 1 --no-cpu > $OUT/bench_D_s2048.log 2>&1 || { tail -20 $OUT/bench_D_s2048.log; exit 1; }
step "bench D default again"
timeout -k 10 300 python bench.py --config D --steps 5 --warmup 1 --no-cpu > $OUT/bench_D2.log 2>&1 || { tail -20 $OUT/bench_D2.log; exit 1; }
step done
