#!/bin/bash
# bench.py under several forward-pass shapes (diagnostic)
cd "$(dirname "$0")/.." && mkdir -p gpurun_out
for s in ${SHAPES:-8,2 8,3 16,1 24,1}; do
GWAMD_POA_LDS_SHAPE=$s timeout -k 10 300 python bench.py --steps 2 --no-cpu > gpurun_out/shape_$s.log 2>&1 || exit 1
done
