#!/bin/bash
# B timing per forward shape (GWAMD_POA_LDS_SHAPE), quick parity on the shape tests
cd "$(dirname "$0")/.." || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/shape_${TAG:-x}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_poa_gpu.py -m gpu -x -q -k "shapes or persistent" --timeout 150 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -2 $O/pytest.log
[ $rc -ne 0 ] && exit $rc
for SH in ${SHAPES:-"8,2" "4,4"}; do
  GWAMD_POA_LDS_SHAPE=$SH timeout -k 10 200 python -u bench.py --config B --steps 10 --warmup 2 --no-cpu > $O/bench_B_$SH.log 2>&1 || { tail -20 $O/bench_B_$SH.log; exit 1; }
  tail -1 $O/bench_B_$SH.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['config']; print('$SH', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], c['grid_slots'], c['phase_ms_mean_per_window'], d['parity']['bit_exact_vs_oracle'])"
done
