#!/bin/bash
# Kernel trace of the driver's bench window (--warmup 5 --steps 20) with t0/t1
# markers, and the kernel timeline inside the timed region.
set -u
export TMPDIR=/tmp
O=gpurun_out/prof_short
rm -rf $O; mkdir -p $O
BENCH_MARKERS=1 timeout -k 10 400 rocprofv3 --kernel-trace ${TRACE_OPTS:-} --output-format csv -d $O -o run -- \
  python bench.py --warmup 5 --steps 20 --no-cpu-baseline --no-eval ${BENCH_ARGS:-} > $O/bench.log 2>&1 \
  || { echo "trace rc=$?"; tail $O/bench.log; exit 3; }
python tools/check_timed_window.py $O $O/timed_window.json > $O/tw.txt
tail -1 $O/bench.log | cut -c1-200
