#!/bin/bash
# round 5: banded Myers waves per launch (parity of the banded aligner tests)
cd "$(dirname "$0")/../.." || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/r5ap
mkdir -p $OUT
echo "[$(date +%T)] pytest banded"
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_aligner_gpu.py tests/test_aligner_long.py tests/test_overlap_align.py -k "banded or Banded or spec or overlap" > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
for C in D_banded D_banded_64k; do
  echo "[$(date +%T)] bench $C"
  timeout -k 10 300 python bench.py --config $C --steps 3 --warmup 1 --no-cpu > $OUT/bench_$C.log 2>&1 || { tail -20 $OUT/bench_$C.log; exit 1; }
done
echo "[$(date +%T)] done"
