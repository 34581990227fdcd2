#!/bin/bash
# Fused-path tests, the driver's short bench line, a default bench line (with the
# CPU baseline), and a marked kernel trace of the short line (timed-window check).
set -u
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q -p no:cacheprovider --timeout 200 --timeout-method thread \
  tests/test_gpu_e2e.py tests/test_gpu_distributed.py > $OUT/e2e.log 2>&1 || { echo "e2e rc=$?"; tail -30 $OUT/e2e.log; exit 3; }
tail -2 $OUT/e2e.log
timeout -k 10 300 python bench.py --warmup 5 --steps 20 --no-cpu-baseline > $OUT/bench_short.log 2>&1 || { echo "short rc=$?"; tail $OUT/bench_short.log; exit 3; }
tail -1 $OUT/bench_short.log | cut -c1-400
BENCH_MARKERS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_short -o run -- \
  python bench.py --warmup 5 --steps 20 --no-cpu-baseline --no-eval > $OUT/prof_short.log 2>&1 || { echo "prof rc=$?"; exit 3; }
python tools/check_timed_window.py $OUT/prof_short $OUT/timed_window_short.json | head -30
timeout -k 10 600 python bench.py > $OUT/bench_default.log 2>&1 || { echo "default rc=$?"; tail $OUT/bench_default.log; exit 3; }
tail -1 $OUT/bench_default.log | cut -c1-400
