#!/bin/bash
# round 5: banded traceback counters (lib/bandprof: tile-staging cycles,
# refills, steps, traceback cycles in the phase slots) on C, B_banded and
# B_banded_1024
cd "$(dirname "$0")/../.." || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/${TAG:-r5bd}
mkdir -p $OUT
for C in C B_banded B_banded_1024; do
  echo "[$(date +%T)] $C"
  GWAMD_DIAG=1 GWAMD_LIBRARY=$PWD/claragenomicsanalysis_amd/lib/bandprof/libgwamd.so timeout -k 10 300 python bench.py --config $C --steps 2 --warmup 1 --no-cpu > $OUT/bench_$C.log 2>&1 || { tail -20 $OUT/bench_$C.log; exit 1; }
  python3 - $OUT/bench_$C.log <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith('{'):
        d = json.loads(l); c = d['config']
        print(d['value'], json.dumps(c.get('phase_ms_mean_per_window')))
PY
done
echo "[$(date +%T)] done"
