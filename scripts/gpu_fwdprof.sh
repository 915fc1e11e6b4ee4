#!/bin/bash
# forward-pass section timers of wave 0 and wave 1 (diagnostic builds), config B.
# Sections (1e5 cycles per window): prefetch = row program records of rows r+2/r+3,
# sig = substitution profile, pred1 = first predecessor + diag/vertical, multi+prefix,
# scan+carry, feed, codes+stores, rest.
cd "$(dirname "$0")/.." || exit 1
O=gpurun_out/fwdprof_${TAG:-x}
mkdir -p $O
for L in prof prof1; do
  GWAMD_DIAG=1 GWAMD_LIBRARY=claragenomicsanalysis_amd/lib/$L/libgwamd.so timeout -k 10 200 python -u bench.py --config B --steps 2 --warmup 1 --no-cpu > $O/$L.log 2>&1 || { tail -5 $O/$L.log; exit 1; }
  tail -1 $O/$L.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); p=d['config']['phase_ms_mean_per_window']; print('$L', 'kernel_ms', d['roofline']['kernel_ms'], 'prefetch', p['forward'], 'sig', p['traceback'], 'pred1', p['rowprog'], 'multi+prefix', p['backbone'], 'scan+carry', p['add'], 'feed', p['topsort'], 'codes+stores', p['output'], 'rest', p['total'])"
done
