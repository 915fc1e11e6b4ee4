#!/bin/bash
# round 2: GPU tests, E bench, default bench line
cd "$(dirname "$0")/.." || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r2a
mkdir -p $O
echo "[$(date +%T)] pytest"
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -5 $O/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
echo "[$(date +%T)] bench E"
timeout -k 10 240 python -u bench.py --config E --steps 8 --warmup 1 > $O/bench_E.log 2>&1 || { tail -20 $O/bench_E.log; exit 1; }
tail -1 $O/bench_E.log | cut -c1-1500
echo "[$(date +%T)] bench default"
timeout -k 10 500 python -u bench.py --steps 20 --warmup 3 > $O/bench_default.log 2>&1 || { tail -20 $O/bench_default.log; exit 1; }
tail -1 $O/bench_default.log | cut -c1-3000
echo "[$(date +%T)] done"
