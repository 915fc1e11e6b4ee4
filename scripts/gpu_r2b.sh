#!/bin/bash
# round 2: CLI order tests, profiles (trace + HBM) and SQ counter passes for B, C, D; trace of E
cd "$(dirname "$0")/.." || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r2b
mkdir -p $O
echo "[$(date +%T)] cli tests"
timeout -k 10 300 python -u -m pytest tests/test_cudapoa_cli.py tests/test_alignment_format.py -m "gpu or not gpu" -x -q --timeout 150 --timeout-method thread > $O/pytest_cli.log 2>&1; rc=$?
tail -3 $O/pytest_cli.log
[ $rc -ne 0 ] && exit $rc
echo "[$(date +%T)] profile B"
TAG=r2_B BENCH_ARGS="--config B --steps 2 --warmup 1 --no-cpu" bash scripts/profile.sh > $O/prof_B.log 2>&1 || { tail -20 $O/prof_B.log; exit 1; }
echo "[$(date +%T)] sq B"
TAG=r2_B BENCH_ARGS="--config B --steps 1 --warmup 0 --no-cpu" bash scripts/pmc_sq.sh > $O/sq_B.log 2>&1 || { tail -20 $O/sq_B.log; exit 1; }
echo "[$(date +%T)] profile C"
TAG=r2_C BENCH_ARGS="--config C --steps 1 --warmup 1 --no-cpu" bash scripts/profile.sh > $O/prof_C.log 2>&1 || { tail -20 $O/prof_C.log; exit 1; }
echo "[$(date +%T)] sq C"
TAG=r2_C BENCH_ARGS="--config C --steps 1 --warmup 0 --no-cpu" bash scripts/pmc_sq.sh > $O/sq_C.log 2>&1 || { tail -20 $O/sq_C.log; exit 1; }
echo "[$(date +%T)] sq D"
TAG=r2_D BENCH_ARGS="--config D --steps 1 --warmup 0 --no-cpu" bash scripts/pmc_sq.sh > $O/sq_D.log 2>&1 || { tail -20 $O/sq_D.log; exit 1; }
echo "[$(date +%T)] trace E"
TAG=r2_E COUNTERS=" " BENCH_ARGS="--config E --steps 4 --warmup 0 --no-cpu" bash scripts/profile.sh > $O/prof_E.log 2>&1 || { tail -20 $O/prof_E.log; exit 1; }
echo "[$(date +%T)] done"
