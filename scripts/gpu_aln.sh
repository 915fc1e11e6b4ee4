#!/bin/bash
# aligner parity tests, Hirschberg-Myers phase profile, config D bench line
cd "$(dirname "$0")/.." || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/aln_${TAG:-x}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_aligner_gpu.py tests/test_overlap_align.py -m gpu -x -q --timeout 150 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python scripts/aln_prof.py 20000 > $O/alnprof.log 2>&1 || { tail -5 $O/alnprof.log; exit 1; }
cat $O/alnprof.log
timeout -k 10 300 python -u bench.py --config D --steps 3 --warmup 1 > $O/bench_D.log 2>&1 || { tail -5 $O/bench_D.log; exit 1; }
tail -1 $O/bench_D.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('D', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['parity'], d['cpu_baseline'] and d['cpu_baseline']['matches_gpu'])"
