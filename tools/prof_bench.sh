#!/bin/bash
# rocprofv3 kernel-trace + stats of a short bench run -> gpurun_out/prof/
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- \
  python bench.py --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/prof/bench.log 2>&1
rc=$?
echo "rc=$rc"; tail -3 gpurun_out/prof/bench.log
find gpurun_out/prof -name "*stats*" | head
exit $rc
