#!/bin/bash
# forward-pass section timers (diagnostic build, see FwdProf) + plain runs
cd "$(dirname "$0")/.." && mkdir -p gpurun_out
for s in ${SHAPES:-24,1 8,3 8,2}; do
GWAMD_POA_LDS_SHAPE=$s GWAMD_DIAG=1 GWAMD_LIBRARY=claragenomicsanalysis_amd/lib/prof/libgwamd.so timeout -k 10 300 python bench.py --steps 2 --no-cpu > gpurun_out/fp_$s.log 2>&1 || exit 1
done
