#!/bin/bash
# Round 4: first GPU check of the round-4 forward pass of the LDS kernel
# (poa_fwd2.hpp): POA parity tests, then config B with the new pass and with
# the round-3 pass (GWAMD_POA_FWD=v1) on the same box.
cd "$(dirname "$0")/.." || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/r4b
mkdir -p $OUT
step() { echo "[$(date +%T)] $*"; }
step "pytest poa gpu"
timeout -k 10 600 python -u -m pytest tests/test_poa_gpu.py tests/test_poa_multibatch.py -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/pytest_poa.log 2>&1 || { tail -30 $OUT/pytest_poa.log; exit 1; }
tail -3 $OUT/pytest_poa.log
step "bench B v2"
timeout -k 10 300 python bench.py --config B --steps 10 --warmup 2 --no-cpu > $OUT/bench_B_v2.log 2>&1 || { tail -20 $OUT/bench_B_v2.log; exit 1; }
step "bench B v1"
GWAMD_DIAG=1 GWAMD_POA_FWD=v1 timeout -k 10 300 python bench.py --config B --steps 10 --warmup 2 --no-cpu > $OUT/bench_B_v1.log 2>&1 || { tail -20 $OUT/bench_B_v1.log; exit 1; }
step done
