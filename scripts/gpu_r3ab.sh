#!/bin/bash
# Round 3: racon DFS sort emitting on the second visit of a stack slot
# (lib/dfx) -- POA parity tests with it, then C and B_msa-style runs A/B.
cd "$(dirname "$0")/.." || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/r3ab
mkdir -p $OUT
step() { echo "[$(date +%T)] $*"; }
step "parity, dfx variant"
GWAMD_LIBRARY=claragenomicsanalysis_amd/lib/dfx/libgwamd.so timeout -k 10 600 python -u -m pytest tests/test_poa_gpu.py tests/test_poa_multibatch.py tests/test_cudapoa_cli.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_dfx.log 2>&1 || { tail -30 $OUT/pytest_dfx.log; exit 1; }
tail -2 $OUT/pytest_dfx.log
for i in 1 2; do
  step "bench C default ($i)"
  timeout -k 10 300 python bench.py --config C --steps 5 --warmup 1 --no-cpu --no-secondary > $OUT/bench_C_def_$i.log 2>&1 || { tail -20 $OUT/bench_C_def_$i.log; exit 1; }
  step "bench C dfx ($i)"
  GWAMD_LIBRARY=claragenomicsanalysis_amd/lib/dfx/libgwamd.so timeout -k 10 300 python bench.py --config C --steps 5 --warmup 1 --no-cpu --no-secondary > $OUT/bench_C_dfx_$i.log 2>&1 || { tail -20 $OUT/bench_C_dfx_$i.log; exit 1; }
done
step done
