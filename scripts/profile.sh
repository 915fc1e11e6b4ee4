#!/bin/bash
# rocprofv3 evidence for bench.py: kernel-trace stats pass, then one PMC pass
# per counter (FETCH_SIZE, WRITE_SIZE), each in its own run (no --pmc with
# trace domains).  Output under gpurun_out/prof_<tag>/.
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
TAG=${TAG:-r1}
ARGS=${BENCH_ARGS:---steps 2 --warmup 1 --no-cpu}
OUT=$ROOT/gpurun_out/prof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp || exit 1
timeout -k 10 ${PROF_TIMEOUT:-420} rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o trace -- python3 $ROOT/bench.py $ARGS > $OUT/trace.log 2>&1 || { echo "trace pass failed"; tail -20 $OUT/trace.log; exit 1; }
tail -2 $OUT/trace.log
for C in ${COUNTERS:-FETCH_SIZE WRITE_SIZE}; do
  timeout -k 10 ${PROF_TIMEOUT:-420} rocprofv3 --pmc $C --output-format csv -d $OUT/pmc_$C -o pmc -- python3 $ROOT/bench.py $ARGS > $OUT/pmc_$C.log 2>&1 || { echo "pmc $C failed"; tail -20 $OUT/pmc_$C.log; exit 1; }
done
find $OUT -name "*.csv" | head -20
