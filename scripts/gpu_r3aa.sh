#!/bin/bash
# Round 3: forward pass inlined (default) vs called (lib/noinl), and the Kahn
# sort with the successor list read ahead (lib/tsx), configs B and C, A/B on
# one box; parity of both variants on the POA GPU tests.
cd "$(dirname "$0")/.." || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/r3aa
mkdir -p $OUT
step() { echo "[$(date +%T)] $*"; }
for i in 1 2; do
  step "bench B inlined ($i)"
  timeout -k 10 300 python bench.py --config B --steps 5 --warmup 1 --no-cpu --no-secondary > $OUT/bench_B_inl_$i.log 2>&1 || { tail -20 $OUT/bench_B_inl_$i.log; exit 1; }
  step "bench B called ($i)"
  GWAMD_LIBRARY=claragenomicsanalysis_amd/lib/noinl/libgwamd.so timeout -k 10 300 python bench.py --config B --steps 5 --warmup 1 --no-cpu --no-secondary > $OUT/bench_B_noinl_$i.log 2>&1 || { tail -20 $OUT/bench_B_noinl_$i.log; exit 1; }
done
for i in 1 2; do
  for C in B C; do
    step "bench $C default ($i)"
    timeout -k 10 300 python bench.py --config $C --steps 5 --warmup 1 --no-cpu --no-secondary > $OUT/bench_${C}_def_$i.log 2>&1 || { tail -20 $OUT/bench_${C}_def_$i.log; exit 1; }
    step "bench $C tsx ($i)"
    GWAMD_LIBRARY=claragenomicsanalysis_amd/lib/tsx/libgwamd.so timeout -k 10 300 python bench.py --config $C --steps 5 --warmup 1 --no-cpu --no-secondary > $OUT/bench_${C}_tsx_$i.log 2>&1 || { tail -20 $OUT/bench_${C}_tsx_$i.log; exit 1; }
  done
done
step "parity, tsx variant"
GWAMD_LIBRARY=claragenomicsanalysis_amd/lib/tsx/libgwamd.so timeout -k 10 600 python -u -m pytest tests/test_poa_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_tsx.log 2>&1 || { tail -30 $OUT/pytest_tsx.log; exit 1; }
tail -2 $OUT/pytest_tsx.log
step "parity, called variant"
GWAMD_LIBRARY=claragenomicsanalysis_amd/lib/noinl/libgwamd.so timeout -k 10 600 python -u -m pytest tests/test_poa_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_noinl.log 2>&1 || { tail -30 $OUT/pytest_noinl.log; exit 1; }
tail -2 $OUT/pytest_noinl.log
step done
