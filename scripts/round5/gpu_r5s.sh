#!/bin/bash
# round 5: band kernel past 512 with a 32-row traceback tile (8-row ring at
# 1,024): four windows per CU (parity, benches)
cd "$(dirname "$0")/../.." || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/${TAG:-r5s}
mkdir -p $OUT
echo "[$(date +%T)] pytest banded poa"
[ -n "$SKIP_TESTS" ] || timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_poa_gpu.py tests/test_poa_weights.py -k "band or Band" > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
[ -n "$SKIP_TESTS" ] || tail -2 $OUT/pytest.log
for C in B_banded_1024 B_banded_384 B_banded_512 B_banded C; do
  echo "[$(date +%T)] bench $C"
  timeout -k 10 300 python bench.py --config $C --steps 3 --warmup 1 --no-cpu > $OUT/bench_$C.log 2>&1 || { tail -20 $OUT/bench_$C.log; exit 1; }
done
echo "[$(date +%T)] done"
