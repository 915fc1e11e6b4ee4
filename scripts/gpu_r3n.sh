#!/bin/bash
# Round 3, call n: section counters of the parallel add on config C.
cd "$(dirname "$0")/.." || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/r3n
mkdir -p $OUT
step() { echo "[$(date +%T)] $*"; }
step "C addprof"
GWAMD_LIBRARY=$PWD/claragenomicsanalysis_amd/lib/addprof/libgwamd.so timeout -k 10 300 python bench.py --config C --steps 1 --warmup 0 --no-cpu --no-secondary > $OUT/bench_C_addprof.log 2>&1 || { tail -20 $OUT/bench_C_addprof.log; exit 1; }
python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d['config'].get('phase_ms_mean_per_window'))" $OUT/bench_C_addprof.log
step done
