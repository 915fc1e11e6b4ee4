#!/bin/bash
# round 5: Kahn pop without exec-masked successor loads (lanes past the count
# repeat the last successor) and an untested next-word read with all queued
# words: topsort / parity tests, then C, B and F_int32_4k with phase splits
cd "$(dirname "$0")/../.." || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/${TAG:-r5bc}
mkdir -p $OUT
echo "[$(date +%T)] tests"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "topsort or full_parity or banded_parity or config_c or anti_diagonal or kat" > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
for C in ${CONFIGS:-B C F_int32_4k B_banded}; do
  echo "[$(date +%T)] $C"
  timeout -k 10 300 python bench.py --config $C --steps 3 --warmup 1 --no-cpu > $OUT/bench_$C.log 2>&1 || { tail -20 $OUT/bench_$C.log; exit 1; }
  python3 - $OUT/bench_$C.log <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith('{'):
        d = json.loads(l); c = d['config']
        print(d['value'], d['ms_per_step'], d['roofline'].get('kernel_ms'), json.dumps(c.get('phase_ms_mean_per_window')))
PY
done
echo "[$(date +%T)] done"
