# round 6: aligner parity after the run-ahead change, the
# bench lines they move and the D_banded_64k profile
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/${TAG:-r6b}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_aligner_long.py tests/test_aligner_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
for C in ${LINES:-D_banded_64k D_ukkonen_64k D_ukkonen}; do
  timeout -k 10 400 python bench.py --config $C --steps 3 --warmup 1 > $OUT/bench_$C.log 2>&1 || { tail -20 $OUT/bench_$C.log; exit 1; }
  tail -c 1200 $OUT/bench_$C.log
done
for C in ${PROFILE:-D_banded_64k}; do
  TAG=${TAG:-r6b}_$C PROF_TIMEOUT=300 BENCH_ARGS="--config $C --steps 2 --warmup 1 --no-cpu --no-secondary" bash scripts/profile.sh > $OUT/prof_$C.log 2>&1 || { tail -20 $OUT/prof_$C.log; exit 1; }
done
echo done
