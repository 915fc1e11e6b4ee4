#!/bin/bash
# Round 4: banded Myers default tile now min(2 KiB, whole-query state):
# aligner parity, then D_banded and D_banded_64k default lines.
cd "$(dirname "$0")/.." || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/r4p
mkdir -p $OUT
step() { echo "[$(date +%T)] $*"; }
step "pytest aligner"
timeout -k 10 600 python -u -m pytest tests/test_aligner_gpu.py tests/test_aligner_long.py -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_aln.log 2>&1 || { tail -30 $OUT/pytest_aln.log; exit 1; }
tail -2 $OUT/pytest_aln.log
step "bench D_banded"
timeout -k 10 300 python bench.py --config D_banded --steps 5 --warmup 1 > $OUT/bench_D_banded.log 2>&1 || { tail -20 $OUT/bench_D_banded.log; exit 1; }
step "bench D_banded_64k"
timeout -k 10 300 python bench.py --config D_banded_64k --steps 3 --warmup 1 --no-cpu > $OUT/bench_D_banded_64k.log 2>&1 || { tail -20 $OUT/bench_D_banded_64k.log; exit 1; }
step done
