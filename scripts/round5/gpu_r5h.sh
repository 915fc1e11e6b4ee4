#!/bin/bash
# round 5: the LDS kernel's forward pass without the per-row vmcnt(0) wait
# (ring mask and list pointer out of the flat RowProg): POA parity, then B, E, F
cd "$(dirname "$0")/../.." || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/r5h
mkdir -p $OUT
echo "[$(date +%T)] pytest poa"
timeout -k 10 900 python -u -m pytest tests/test_poa_gpu.py tests/test_poa_weights.py tests/test_poa_multibatch.py -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_poa.log 2>&1 || { tail -40 $OUT/pytest_poa.log; exit 1; }
tail -2 $OUT/pytest_poa.log
for C in B F_int32_4k B_banded; do
  echo "[$(date +%T)] bench $C"
  timeout -k 10 300 python bench.py --config $C --steps 5 --warmup 1 --no-cpu > $OUT/bench_$C.log 2>&1 || { tail -20 $OUT/bench_$C.log; exit 1; }
done
echo "[$(date +%T)] bench E"
timeout -k 10 300 python bench.py --config E --steps 10 --warmup 1 --no-cpu > $OUT/bench_E.log 2>&1 || { tail -20 $OUT/bench_E.log; exit 1; }
echo "[$(date +%T)] done"
