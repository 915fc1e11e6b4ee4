#!/bin/bash
# Round 3, call j: short Hirschberg-Myers with its query patterns in HBM
# (GWAMD_HM_PAT_HBM=1, hm_kernel<2>): aligner parity with the knob set, then
# config D with and without it.
cd "$(dirname "$0")/.." || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/r3j
mkdir -p $OUT
step() { echo "[$(date +%T)] $*"; }
step "pytest aligner with pattern HBM"
GWAMD_HM_PAT_HBM=1 timeout -k 10 400 python -u -m pytest tests/test_aligner_gpu.py tests/test_aligner_long.py -m gpu -x -v --timeout 150 --timeout-method thread > $OUT/pytest_pat.log 2>&1 || { tail -30 $OUT/pytest_pat.log; exit 1; }
tail -2 $OUT/pytest_pat.log
for K in 0 1 0 1; do
  step "bench D pat_hbm=$K"
  GWAMD_HM_PAT_HBM=$K timeout -k 10 300 python bench.py --config D --steps 3 --warmup 1 --no-cpu > $OUT/bench_D_$K.log 2>&1 || { tail -20 $OUT/bench_D_$K.log; exit 1; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d.get('roofline',{}).get('frac'))" $OUT/bench_D_$K.log
done
step done
