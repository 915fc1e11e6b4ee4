#!/bin/bash
# round 5: config D with the pipelined align_all (and one-stage for A/B),
# config C without the anti-diagonal pass's code stores (timing experiment)
cd "$(dirname "$0")/../.." || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/r5e
mkdir -p $OUT
echo "[$(date +%T)] bench D"
timeout -k 10 300 python bench.py --config D --steps 3 --warmup 1 --no-cpu > $OUT/bench_D.log 2>&1 || { tail -20 $OUT/bench_D.log; exit 1; }
echo "[$(date +%T)] bench D one-stage"
GWAMD_DIAG=1 GWAMD_ALIGNER_PIPELINE=0 timeout -k 10 300 python bench.py --config D --steps 3 --warmup 1 --no-cpu > $OUT/bench_D_1stage.log 2>&1 || { tail -20 $OUT/bench_D_1stage.log; exit 1; }
echo "[$(date +%T)] C nocode"
GWAMD_DIAG=1 GWAMD_LIBRARY=claragenomicsanalysis_amd/lib/exp1/libgwamd.so timeout -k 10 300 python bench.py --config C --steps 2 --warmup 1 --no-cpu > $OUT/bench_C_nocode.log 2>&1
rc=$?; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then tail -20 $OUT/bench_C_nocode.log; exit 1; fi
echo "[$(date +%T)] done"
