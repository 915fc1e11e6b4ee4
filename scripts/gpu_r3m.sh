#!/bin/bash
# Round 3, call m: parallel add changes (all POA
# kernels): the whole GPU suite, then the B, C and B_banded lines.
cd "$(dirname "$0")/.." || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/r3m
mkdir -p $OUT
step() { echo "[$(date +%T)] $*"; }
step "pytest -m gpu"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
for C in C B B_banded; do
  step "bench $C"
  timeout -k 10 300 python bench.py --config $C --steps 3 --warmup 1 --no-cpu --no-secondary > $OUT/bench_$C.log 2>&1 || { tail -20 $OUT/bench_$C.log; exit 1; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['parity'].get('bit_exact_vs_oracle'), d['config'].get('phase_ms_mean_per_window'))" $OUT/bench_$C.log
done
step done
