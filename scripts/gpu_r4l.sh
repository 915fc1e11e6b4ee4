#!/bin/bash
# Round 4: hm_kernel at 4 waves per SIMD (amdgpu_waves_per_eu(4): 120 VGPRs
# instead of 152): aligner parity, then the D line.
cd "$(dirname "$0")/.." || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/r4l
mkdir -p $OUT
step() { echo "[$(date +%T)] $*"; }
step "pytest aligner"
timeout -k 10 600 python -u -m pytest tests/test_aligner_gpu.py tests/test_aligner_long.py -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_aln.log 2>&1 || { tail -30 $OUT/pytest_aln.log; exit 1; }
tail -2 $OUT/pytest_aln.log
for i in 1 2; do
step "bench D $i"
timeout -k 10 300 python bench.py --config D --steps 5 --warmup 1 --no-cpu > $OUT/bench_D$i.log 2>&1 || { tail -20 $OUT/bench_D$i.log; exit 1; }
done
step done
