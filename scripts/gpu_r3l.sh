#!/bin/bash
# Round 3, call l: real-row spill rule (only far rows and rows that are not real
# hold values <= Tmax: banded parity tests, then C and B_banded lines, the C
# kernel trace and HBM passes.
cd "$(dirname "$0")/.." || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/r3l
mkdir -p $OUT
step() { echo "[$(date +%T)] $*"; }
step "pytest banded"
timeout -k 10 600 python -u -m pytest tests/test_poa_gpu.py tests/test_poa_multibatch.py -m gpu -x -v -k "band or msa or C" --timeout 150 --timeout-method thread > $OUT/pytest_band.log 2>&1 || { tail -30 $OUT/pytest_band.log; exit 1; }
tail -2 $OUT/pytest_band.log
for C in C C B_banded B_banded_512; do
  step "bench $C"
  timeout -k 10 300 python bench.py --config $C --steps 3 --warmup 1 --no-cpu > $OUT/bench_$C.log 2>&1 || { tail -20 $OUT/bench_$C.log; exit 1; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['parity'].get('bit_exact_vs_oracle'), d['config'].get('phase_ms_mean_per_window'))" $OUT/bench_$C.log
done
step "profile C"
TAG=r3l_C PROF_TIMEOUT=300 BENCH_ARGS="--config C --steps 1 --warmup 1 --no-cpu --no-secondary" bash scripts/profile.sh > $OUT/prof_C.log 2>&1 || { tail -20 $OUT/prof_C.log; exit 1; }
step done
