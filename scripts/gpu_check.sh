#!/bin/bash
# GPU-box check: parity tests, smoke, then a short bench.  Stops at the first
# fault/abort/timeout (exit codes other than 0/1 from pytest).
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 ${TEST_TIMEOUT:-600} python -m pytest tests -m gpu -q ${PYTEST_ARGS} > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -30 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
if [ -n "$SKIP_BENCH" ]; then exit $rc; fi
timeout -k 10 ${BENCH_TIMEOUT:-600} python bench.py ${BENCH_ARGS} > gpurun_out/bench.log 2>&1
brc=$?
tail -5 gpurun_out/bench.log
exit $brc
