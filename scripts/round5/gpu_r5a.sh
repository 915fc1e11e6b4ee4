#!/bin/bash
# round 5: new parity tests (weights, marked rows, wide Ukkonen 3-4 rows per
# thread, aligner stats), then config E with 2 pinned CPUs against unpinned
cd "$(dirname "$0")/../.." || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/r5a
mkdir -p $OUT
step() { echo "[$(date +%T)] $*"; }
step "pytest new"
timeout -k 10 900 python -u -m pytest tests/test_poa_weights.py "tests/test_poa_gpu.py::test_marked_rows_multi_source_fwd2" "tests/test_aligner_long.py::test_ukkonen_wide_band_matches_oracle" tests/test_aligner_gpu.py -m gpu -v --timeout 300 --timeout-method thread > $OUT/pytest_new.log 2>&1
rc=$?
tail -30 $OUT/pytest_new.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
step "E unpinned"
timeout -k 10 300 python bench.py --config E --steps 10 --warmup 1 --no-cpu > $OUT/bench_E.log 2>&1 || { tail -20 $OUT/bench_E.log; exit 1; }
step "E 2 cpus"
timeout -k 10 300 python bench.py --config E --steps 10 --warmup 1 --no-cpu --cpus 2 > $OUT/bench_E_cpus2.log 2>&1 || { tail -20 $OUT/bench_E_cpus2.log; exit 1; }
step "E 4 cpus"
timeout -k 10 300 python bench.py --config E --steps 10 --warmup 1 --no-cpu --cpus 4 > $OUT/bench_E_cpus4.log 2>&1 || { tail -20 $OUT/bench_E_cpus4.log; exit 1; }
step done
