#!/bin/bash
# Round 4: banded Myers chunk state in LDS up to 160 KiB, multi-wave sweep: long-pair parity,
# then the D_banded_64k and D_banded lines.
cd "$(dirname "$0")/.." || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/r4g
mkdir -p $OUT
step() { echo "[$(date +%T)] $*"; }
step "pytest aligner long"
timeout -k 10 600 python -u -m pytest tests/test_aligner_long.py tests/test_aligner_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_aln.log 2>&1 || { tail -30 $OUT/pytest_aln.log; exit 1; }
tail -2 $OUT/pytest_aln.log
for C in D_banded_64k D_banded; do
  step "bench $C"
  timeout -k 10 300 python bench.py --config $C --steps 2 --warmup 1 --no-cpu > $OUT/bench_$C.log 2>&1 || { tail -20 $OUT/bench_$C.log; exit 1; }
done
step done
