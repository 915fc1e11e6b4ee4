#!/bin/bash
# round 5: full Myers backtrace in 8 x 8 windows (parity, bench, phase counters)
cd "$(dirname "$0")/../.." || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/r5ai
mkdir -p $OUT
echo "[$(date +%T)] pytest myers"
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_aligner_gpu.py tests/test_aligner_long.py tests/test_overlap_align.py -k "myers and not banded and not hirschberg" > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
echo "[$(date +%T)] bench D_myers"
timeout -k 10 300 python bench.py --config D_myers --steps 3 --warmup 1 --no-cpu > $OUT/bench_D_myers.log 2>&1 || { tail -20 $OUT/bench_D_myers.log; exit 1; }
echo "[$(date +%T)] aln_prof myers"
timeout -k 10 300 python scripts/aln_prof.py 20000 myers > $OUT/aln_prof_myers.log 2>&1 || { tail -20 $OUT/aln_prof_myers.log; exit 1; }
tail -8 $OUT/aln_prof_myers.log
echo "[$(date +%T)] done"
