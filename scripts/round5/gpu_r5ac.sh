#!/bin/bash
# round 5: Ukkonen large-tile long-pair parity
cd "$(dirname "$0")/../.." || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/r5ac
mkdir -p $OUT
echo "[$(date +%T)] pytest"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_aligner_long.py -k "ukkonen" > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
echo "[$(date +%T)] done"
