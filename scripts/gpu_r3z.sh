#!/bin/bash
# Round 3: config E stream shape sweep (concurrent batches x windows per batch).
cd "$(dirname "$0")/.." || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/r3z
mkdir -p $OUT
step() { echo "[$(date +%T)] $*"; }
for NB in 2 3 4; do
  for BW in 2048 4096 8192; do
    step "E batches $NB x $BW"
    timeout -k 10 300 python bench.py --config E --steps 8 --warmup 1 --no-cpu --stream-batches $NB --stream-batch-windows $BW > $OUT/E_${NB}_${BW}.log 2>&1 || { tail -20 $OUT/E_${NB}_${BW}.log; exit 1; }
  done
done
step done
