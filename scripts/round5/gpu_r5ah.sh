#!/bin/bash
# round 5: full Myers phase counters (score matrix / backtrace cycles)
cd "$(dirname "$0")/../.." || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/${TAG:-r5ah}
mkdir -p $OUT
echo "[$(date +%T)] aln_prof myers"
timeout -k 10 300 python scripts/aln_prof.py 20000 ${ALGO:-myers} > $OUT/aln_prof_${ALGO:-myers}.log 2>&1 || { tail -20 $OUT/aln_prof_${ALGO:-myers}.log; exit 1; }
tail -14 $OUT/aln_prof_${ALGO:-myers}.log
echo "[$(date +%T)] done"
