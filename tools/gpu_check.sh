#!/bin/bash
# One GPU session: smoke -> GPU parity tests -> short bench. Each GPU step has
# its own time limit; a crash / fault / timeout (exit other than 0 or 1) ends
# the script so nothing else touches the GPU after it.
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
  tail -5 $OUT/$name.log | tee -a $OUT/summary.txt
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "ABORT after $name (rc=$rc)" | tee -a $OUT/summary.txt; exit $rc; fi
  return 0
}
rm -f $OUT/summary.txt
step smoke 300 python __graft_entry__.py smoke
step gputests 900 python -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300
if [ "${BENCH:-1}" = "1" ]; then
  step bench 900 python bench.py ${BENCH_ARGS:-}
fi
exit 0
