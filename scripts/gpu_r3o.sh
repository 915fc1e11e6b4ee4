#!/bin/bash
# Round 3, call o: banded Myers multi-chunk sweep specialised for LDS state
# (no band-matrix loads, so no store waits): banded parity, D_banded_64k and
# D_banded lines.
cd "$(dirname "$0")/.." || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/r3o
mkdir -p $OUT
step() { echo "[$(date +%T)] $*"; }
step "pytest aligner"
timeout -k 10 600 python -u -m pytest tests/test_aligner_gpu.py tests/test_aligner_long.py -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_aln.log 2>&1 || { tail -30 $OUT/pytest_aln.log; exit 1; }
tail -2 $OUT/pytest_aln.log
for C in D_banded_64k D_banded; do
  step "bench $C"
  timeout -k 10 300 python bench.py --config $C --steps 1 --warmup 1 --no-cpu --no-secondary > $OUT/bench_$C.log 2>&1 || { tail -20 $OUT/bench_$C.log; exit 1; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['parity'])" $OUT/bench_$C.log
done
step done
