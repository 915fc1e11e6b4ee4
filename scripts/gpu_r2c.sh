#!/bin/bash
# round 2: 4x4 forward shape parity + B timing per shape; E after pinned pre-reservation
cd "$(dirname "$0")/.." || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r2c
mkdir -p $O
echo "[$(date +%T)] shape tests"
timeout -k 10 300 python -u -m pytest tests/test_poa_gpu.py -m gpu -x -q -k "shapes or persistent or kernel_variants" --timeout 150 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log
[ $rc -ne 0 ] && exit $rc
for SH in "8,2" "4,4"; do
  echo "[$(date +%T)] bench B shape $SH"
  GWAMD_POA_LDS_SHAPE=$SH timeout -k 10 200 python -u bench.py --config B --steps 10 --warmup 2 --no-cpu > $O/bench_B_$SH.log 2>&1 || { tail -20 $O/bench_B_$SH.log; exit 1; }
  tail -1 $O/bench_B_$SH.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['config']['phase_ms_mean_per_window'], d['parity'])"
done
echo "[$(date +%T)] bench E"
timeout -k 10 200 python -u bench.py --config E --steps 8 --warmup 1 > $O/bench_E.log 2>&1 || { tail -20 $O/bench_E.log; exit 1; }
tail -1 $O/bench_E.log | cut -c1-300
echo "[$(date +%T)] done"
