#!/bin/bash
# One GPU session: smoke -> GPU parity tests -> bench lines -> rocprof kernel trace.
# Each GPU step has its own time limit; a crash / fault / timeout (exit other than
# 0 or 1) ends the script so nothing else touches the GPU after it.
set -u
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
step() {  # name, limit, cmd...
  local name=$1 lim=$2; shift 2
  echo "=== $name" | tee -a $OUT/summary.txt
  timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "rc=$rc" | tee -a $OUT/summary.txt
  tail -5 $OUT/$name.log | cut -c1-400 | tee -a $OUT/summary.txt
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "ABORT after $name (rc=$rc)" | tee -a $OUT/summary.txt; exit $rc; fi
  return 0
}
rm -f $OUT/summary.txt
if [ "${SMOKE:-1}" = "1" ]; then
  step smoke 300 python __graft_entry__.py smoke
fi
if [ "${TESTS:-1}" = "1" ]; then
  step gputests 1000 python -u -m pytest ${TEST_ARGS:-tests} -m gpu -v -p no:cacheprovider \
    --timeout 170 --timeout-method thread
fi
if [ "${BENCH:-1}" = "1" ]; then
  step bench_short 300 python bench.py --warmup 5 --steps 20 ${BENCH_ARGS:-}
  step bench 600 python bench.py ${BENCH_ARGS:-}
fi
if [ "${PROF:-0}" = "1" ]; then
  step prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- \
    python bench.py --no-cpu-baseline ${BENCH_ARGS:-}
fi
exit 0
