#!/bin/bash
# round 5: Ukkonen sweep specialised per live chunk count (parity + benches),
# racon DFS list loads (MSA / SPOA_ACCURATE parity + C)
cd "$(dirname "$0")/../.." || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/r5k
mkdir -p $OUT
echo "[$(date +%T)] pytest aligner + poa msa"
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu \
  tests/test_aligner_gpu.py tests/test_aligner_long.py tests/test_poa_gpu.py -k "ukkonen or Ukkonen or racon or msa or accurate or align" \
  > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
for C in D_ukkonen D_ukkonen_64k D_ukkonen_wide_16k D C; do
  echo "[$(date +%T)] bench $C"
  timeout -k 10 300 python bench.py --config $C --steps 3 --warmup 1 --no-cpu > $OUT/bench_$C.log 2>&1 || { tail -20 $OUT/bench_$C.log; exit 1; }
done
echo "[$(date +%T)] done"
