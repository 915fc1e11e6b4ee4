#!/bin/bash
# round 5: batched backtrace tile refills (banded Myers, Ukkonen): aligner
# parity, the banded / Ukkonen bench lines, and config D's step breakdown
cd "$(dirname "$0")/../.." || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/r5d
mkdir -p $OUT
echo "[$(date +%T)] pytest aligners"
timeout -k 10 900 python -u -m pytest tests/test_aligner_gpu.py tests/test_aligner_long.py -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_aln.log 2>&1 || { tail -40 $OUT/pytest_aln.log; exit 1; }
tail -2 $OUT/pytest_aln.log
for C in D_ukkonen D_banded D_ukkonen_64k D_banded_64k D_ukkonen_wide_16k; do
  echo "[$(date +%T)] bench $C"
  timeout -k 10 400 python bench.py --config $C --steps 3 --warmup 1 > $OUT/bench_$C.log 2>&1 || { tail -20 $OUT/bench_$C.log; exit 1; }
done
echo "[$(date +%T)] D breakdown"
timeout -k 10 300 python scripts/aln_breakdown.py > $OUT/aln_breakdown.log 2>&1 || { tail -20 $OUT/aln_breakdown.log; exit 1; }
cat $OUT/aln_breakdown.log
echo "[$(date +%T)] C phases: default vs no AD code stores"
timeout -k 10 300 python bench.py --config C --steps 2 --warmup 1 --no-cpu > $OUT/bench_C.log 2>&1 || { tail -20 $OUT/bench_C.log; exit 1; }
GWAMD_DIAG=1 GWAMD_LIBRARY=claragenomicsanalysis_amd/lib/exp1/libgwamd.so timeout -k 10 300 python bench.py --config C --steps 2 --warmup 1 --no-cpu > $OUT/bench_C_nocode.log 2>&1
rc=$?; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then tail -20 $OUT/bench_C_nocode.log; exit 1; fi
echo "[$(date +%T)] done"
