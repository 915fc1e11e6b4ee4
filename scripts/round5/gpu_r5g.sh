#!/bin/bash
# round 5: K-stage pipelined align_all (copy-in / copy-out streams): aligner
# parity, then config D and the D_* lines
cd "$(dirname "$0")/../.." || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/r5g
mkdir -p $OUT
echo "[$(date +%T)] pytest aligners"
timeout -k 10 900 python -u -m pytest tests/test_aligner_gpu.py tests/test_overlap_align.py tests/test_alignment_format.py -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_aln.log 2>&1 || { tail -40 $OUT/pytest_aln.log; exit 1; }
tail -2 $OUT/pytest_aln.log
for C in D D_myers D_banded D_ukkonen; do
  echo "[$(date +%T)] bench $C"
  timeout -k 10 300 python bench.py --config $C --steps 3 --warmup 1 --no-cpu > $OUT/bench_$C.log 2>&1 || { tail -20 $OUT/bench_$C.log; exit 1; }
done
for K in 1 2 8; do
  echo "[$(date +%T)] bench D stages $K"
  GWAMD_DIAG=1 GWAMD_ALIGNER_PIPELINE=$K timeout -k 10 300 python bench.py --config D --steps 3 --warmup 1 --no-cpu > $OUT/bench_D_k$K.log 2>&1 || { tail -20 $OUT/bench_D_k$K.log; exit 1; }
done
echo "[$(date +%T)] done"
